"""Stand-alone launch times (HIP events) of the VAE weight gradients at the
train step's T*B = 24,576 rows: the bf16 configuration's seven layers on the
per-layer gemm_bf16 split-K form (the model's split choice) against the
grouped tall-K kernel (wgrad_tn.hip), and the fp32 configuration's four x3
layers on gemm_x3_tn.  Prints one JSON line per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

K = int(os.environ.get("WG_K", 24576))
dev = "cuda:0"
VAE = [(784, 512, 784, 512), (512, 256, 512, 256), (256, 50, 256, 56), (256, 50, 256, 56),
       (50, 256, 56, 256), (256, 512, 256, 512), (512, 784, 512, 784)]
if os.environ.get("WG_PROBS"):  # a subset of the layers
    VAE = [VAE[int(i)] for i in os.environ["WG_PROBS"].split(",")]
torch.manual_seed(0)
Xs = [(torch.randn(K, lda, device=dev) * 0.5).to(torch.bfloat16) for M, N, lda, ldb in VAE]
Ys = [(torch.randn(K, ldb, device=dev) * 0.1).to(torch.bfloat16) for M, N, lda, ldb in VAE]
Cs = [torch.zeros(M, N, device=dev) for M, N, _, _ in VAE]
bs = [torch.zeros(N, device=dev) for _, N, _, _ in VAE]
flops = sum(2.0 * K * M * N for M, N, _, _ in VAE)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def old_layer(i):
    M, N, lda, ldb = VAE[i]
    big = M >= 128 and N >= 128
    tiles = ((M + 127) // 128) * ((N + 127) // 128) if big else ((M + 63) // 64) * ((N + 63) // 64)
    sk = max(1, min(K // 512, (256 + tiles - 1) // tiles))
    ops.gemm_bf16([Xs[i]], [Ys[i]], [Cs[i]], M, N, K, lda, ldb, N, tn=True, epi=ops.BF_ATOMIC,
                  splitk=sk, colsum=[bs[i]])


ONLY_NEW = os.environ.get("WG_ONLY_NEW") == "1"
per = [0.0] if ONLY_NEW else [timeit(lambda i=i: old_layer(i)) for i in range(len(VAE))]
if not ONLY_NEW:
  print(json.dumps({"variant": "gemm_bf16 per layer", "K": K, "us_per_layer": per,
                  "us_total": sum(per), "frac_bf16": flops / (sum(per) * 1e-6) / 2.5e15}))


def new(nsplit):
    ops.wgrad_tn_bf16(Xs, Ys, Cs, bs, [(M, N, lda, ldb, N) for M, N, lda, ldb in VAE], K, nsplit)


ref = [(X.double()[:, :M].t() @ Y.double()[:, :N]) for X, Y, (M, N, _, _) in zip(Xs, Ys, VAE)]
for nsplit in [int(x) for x in os.environ.get("WG_SPLITS", "8,16,4,24").split(",")]:
    for c in Cs:
        c.zero_()
    new(nsplit)
    torch.cuda.synchronize()
    err = max(((c.double() - r).abs().max() / r.abs().max()).item() for c, r in zip(Cs, ref))
    us = timeit(lambda: new(nsplit))
    print(json.dumps({"variant": "wgrad_tn_bf16 grouped", "K": K, "nsplit": nsplit, "us_total": us,
                      "frac_bf16": flops / (us * 1e-6) / 2.5e15, "max_rel_err": err,
                      "mode": os.environ.get("MOG_WG_MODE", "0"),
                      "map": os.environ.get("MOG_WG_MAP", "1"), "probs": os.environ.get("WG_PROBS")}))

if ONLY_NEW:
    sys.exit(0)
# the fp32 configuration's x3 weight gradients (rec1, rec2, gen2, gen_mean)
X3 = [(784, 512), (512, 256), (256, 512), (512, 784)]
Af = [torch.randn(K, M, device=dev) for M, _ in X3]
Bf = [torch.randn(K, N, device=dev) * 0.1 for _, N in X3]
Cf = [torch.zeros(M, N, device=dev) for M, N in X3]
bf = [torch.zeros(N, device=dev) for _, N in X3]
per = []
for i, (M, N) in enumerate(X3):
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    sk = max(1, min(K // 256, (512 + tiles - 1) // tiles))
    per.append(timeit(lambda i=i, M=M, N=N, sk=sk: ops.gemm_x3_tn(
        Af[i], Bf[i], Cf[i], M, N, K, M, N, N, splitk=sk, colsum=bf[i], reduce=False)))
fl3 = sum(2.0 * K * M * N for M, N in X3)
print(json.dumps({"variant": "gemm_x3_tn per layer", "K": K, "us_per_layer": per,
                  "us_total": sum(per), "frac_fp32": fl3 / (sum(per) * 1e-6) / 157.3e12}))
ref3 = [(a.double().t() @ b.double()) for a, b in zip(Af, Bf)]
for nsplit in [int(x) for x in os.environ.get("WG_X3_SPLITS", "8,7,16").split(",")]:
    def go3():
        ops.wgrad_tn_x3(Af, Bf, Cf, bf, [(M, N, M, N, N) for M, N in X3], K, nsplit)
    for c in Cf:
        c.zero_()
    go3()
    torch.cuda.synchronize()
    err = max(((c.double() - r).abs().max() / r.abs().max()).item() for c, r in zip(Cf, ref3))
    us = timeit(go3)
    print(json.dumps({"variant": "wgrad_tn_x3 grouped", "K": K, "nsplit": nsplit, "us_total": us,
                      "frac_fp32": fl3 / (us * 1e-6) / 157.3e12,
                      "frac_bf16_x6": 6 * fl3 / (us * 1e-6) / 2.5e15, "max_rel_err": err}))
