"""Time the fused step kernel with phases masked out (MOG_VS_PHASES bit mask:
1 STN read, 2 dense layers, 8 STN write, 16 activation flushes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mog_air.air_model import AIRModel  # noqa: E402
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    m = AIRModel(max_steps=3, cnn=False, train=True, device="cuda:0", precision="bf16",
                 scope="vs")
    x, k = bench.synthetic(B, 50)
    x = torch.as_tensor(x).to("cuda:0")
    k = torch.as_tensor(k).to("cuda:0")
    m.step(x, k)
    torch.cuda.synchronize()
    ws = m._ws
    masks = [int(v) for v in os.environ.get("VS_MASKS", "31,1,2,8,16,0").split(",")]
    for mask in masks:
        os.environ["MOG_VS_PHASES"] = str(mask)
        for _ in range(3):
            m._step_fused(x, ws, 0, 0.3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        n = 10
        for _ in range(n):
            m._step_fused(x, ws, 0, 0.3)
        e1.record()
        torch.cuda.synchronize()
        print(f"phases {mask:2d}: {e0.elapsed_time(e1) / n * 1e3:8.1f} us", flush=True)


def timing(B):
    """per-phase in-kernel timestamps (MOG_VS_TIMING)"""
    m = AIRModel(max_steps=3, cnn=False, train=True, device="cuda:0", precision="bf16",
                 scope="vst%d" % B)
    x, k = bench.synthetic(B, 51)
    x = torch.as_tensor(x).to("cuda:0")
    k = torch.as_tensor(k).to("cuda:0")
    m.step(x, k)
    torch.cuda.synchronize()
    os.environ["MOG_VS_TIMING"] = "1"
    for t in range(3):
        m._step_fused(x, m._ws, t, 0.3)
    del os.environ["MOG_VS_TIMING"]


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "timing":
        timing(int(sys.argv[1]))
        sys.exit(0)
    main()
