"""The STN read backward launched on the main stream while one candidate
kernel runs on the side stream: mismatching images against the same launch
alone (which is deterministic).  Localises a kernel that corrupts a
co-resident workgroup."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_streams as ts  # noqa: E402
from mog_air import ops  # noqa: E402

B = 1024
data = ts._data(B)
m = ts._air("conc", "fp32")
m.ONE_PASS_WGRADS = True
m.compute_gradients(*data[0])
torch.cuda.synchronize()
ws, W, TB = m._ws, m.windows_size, B * m.max_steps
X = data[0][0].reshape(B, -1)
main = torch.cuda.current_stream()
side = m._side_stream()


VICTIM = os.environ.get("VICTIM", "stn")


def stn(out):
    if VICTIM == "gemm":
        from mog_air.ops import gemm
        gemm([ws.g.view(TB, -1)], [m._P("vae/recognition_1/weights")], [out.view(TB, -1)], TB, 512,
             784, 784, 512, 512)
        return
    ops.stn_backward(X, ws.th_f, (W, W), ws.dg_all, want_dU=False, dtheta=out, n=TB)


ref = torch.empty_like(ws.dth_f_all) if VICTIM == "stn" else torch.empty((TB, 512), device="cuda:0")
stn(ref)
torch.cuda.synchronize()
W2, R1, R2, Z, G1, G2 = m._vae_dims()
scratch = torch.zeros_like(m.params.grad)
sg = lambda n: scratch[m.params.offsets["air/rnn/vae/" + n + "/weights"]:][:m._P("vae/" + n + "/weights").numel()]  # noqa: E731


def x3_tn():
    ops.gemm_x3_tn(ws.g, ws.da1, scratch, W2, R1, TB, W2, R1, R1, splitk=1)


def dw_fp32():
    m._dw(ws.z, ws.dd1, scratch, TB, Z, G1, Z, G1)


def dw_fp32_n50():
    m._dw(ws.a2, ws.dmu, scratch, TB, R2, Z, R2, Z)


Xb = torch.zeros((TB, 784), device="cuda:0", dtype=torch.bfloat16)
Yb = torch.zeros((TB, 512), device="cuda:0", dtype=torch.bfloat16)
Xb.copy_(ws.g.view(TB, -1))
Yb.copy_(ws.da1.view(TB, -1))
Wb = torch.zeros((512, 784), device="cuda:0", dtype=torch.bfloat16)
outb = torch.zeros((TB, 512), device="cuda:0")
X3 = torch.zeros((3, TB, 784), device="cuda:0", dtype=torch.bfloat16)
Y3 = torch.zeros((3, TB, 512), device="cuda:0", dtype=torch.bfloat16)
ops.split3_bf16(ws.g.view(TB, -1), X3, TB, 784, 784, 784, TB * 784)
ops.split3_bf16(ws.da1.view(TB, -1), Y3, TB, 512, 512, 512, TB * 512)
W3 = m._w3()["recognition_1"]


def bf16_tn():
    from mog_air.ops import BF_ATOMIC, gemm_bf16
    gemm_bf16([Xb], [Yb], [scratch], W2, R1, TB, 784, 512, R1, tn=True, epi=BF_ATOMIC, splitk=1)


def bf16_nt():
    from mog_air.ops import BF_STORE, gemm_bf16
    gemm_bf16([Xb], [Wb], [outb], TB, 512, 784, 784, 784, 512, epi=BF_STORE)


def x3p_tn():
    ops.gemm_x3p_tn(X3.view(-1), TB * 784, Y3, TB * 512, scratch, W2, R1, TB, 784, 512, R1, splitk=1)


def x3_nt():
    ops.gemm_x3_nt(ws.da1.view(TB, -1), W3, 784 * 512, outb2, TB, 784, 512, 512, 512, 784)


outb2 = torch.zeros((TB, 784), device="cuda:0")


def heads():
    m._weight_grads_heads(ws)


def spin():
    ops.spin(200000)


def poison():
    ops.lds_poison(0x7FC00000)


CANDS = {"none": None, "spin": spin, "x3_tn": x3_tn, "bf16_tn": bf16_tn, "bf16_nt": bf16_nt,
         "x3p_tn": x3p_tn, "x3_nt": x3_nt, "dw_fp32_g1": dw_fp32, "dw_fp32_n50": dw_fp32_n50,
         "heads_dw": heads, "lds_poison": poison}
only = sys.argv[1:] or list(CANDS)
for name in only:
    fn = CANDS[name]
    bad = []
    for r in range(24):
        out = torch.empty_like(ref)
        if fn is not None:
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                for _ in range(3):
                    fn()
        # stagger: the STN launch lands at different points of the side work
        ops.spin(r * 2000)
        stn(out)
        torch.cuda.synchronize()
        bad.append(int((out.view(TB, -1) != ref.view(TB, -1)).any(dim=1).sum()))
    print(f"{name:12s} mismatching images per launch: {bad}", flush=True)
