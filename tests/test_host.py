"""CPU tests of the host side: the C ABI library loads and exports every
symbol declared in include/*.h (no compute call without a GPU), and the host
logic (parameter table, annealing, -ap prior) restates the reference like the
oracle does."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from mog_air import _lib
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    # every declared symbol has a ctypes signature and vice versa
    assert set(syms) == set(_lib._SIGS)


def test_test_instruments_live_outside_the_product_library():
    """mog_spin / mog_lds_poison (include/mog_air_test.h) are exported by
    libmog_air_test.so only: the product library carries no test kernels."""
    import re
    from mog_air import _lib
    with open(os.path.join(ROOT, "include", "mog_air_test.h")) as f:
        src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    syms = sorted(set(re.findall(r"\bint\s+(mog_\w+)\s*\(", src)))
    assert syms == sorted(_lib._TEST_SIGS)
    test_lib, lib = _lib.load_test(), _lib.load()
    for s in syms:
        assert hasattr(test_lib, s), s
        assert not hasattr(lib, s), s


def test_library_built_from_these_sources():
    """Build provenance: the source hash compiled into libmog_air.so
    (mog_build_id) equals the hash of the sources beside it, which
    _lib.load() checks before any launch (a stale library refuses to load)."""
    from mog_air import _lib
    built = _lib.library_build_id()
    assert len(built) == 16 and built == _lib.source_build_id()


def test_all_headers_symbols_exported():
    """Every include/*.h entry point is exported: the product headers by
    libmog_air.so, include/mog_air_test.h by libmog_air_test.so."""
    from mog_air import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    test_lib = ctypes.CDLL(_lib.TEST_LIB_PATH)
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        src = open(os.path.join(inc, fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for name in re.findall(r"\bint\s+(mog_\w+)\s*\(", src):
            assert hasattr(test_lib if fn == "mog_air_test.h" else lib, name), (fn, name)


def test_torch_ops_extension_registers_every_launch_op():
    """csrc/torch_ops.cpp: the TORCH_LIBRARY fragment loads on a CPU host and
    registers the launch-level ops the AIRModel dispatches through; a CPU
    tensor finds no kernel (no CPU fallback)."""
    from mog_air import _lib
    _lib.load_torch_ops()
    names = ("gemm_f32_", "gemm_f32_kseg_", "gemm_bf16_", "cvt_bf16_batch_", "stn_forward_",
             "stn_backward_", "stn_backward_sigmoid_", "lstm_cell_forward_",
             "lstm_cell_backward_", "lstm_cell_forward2_", "lstm_cell_backward2_", "gemm_f32_kseg_group_",
             "air_step_forward_", "air_step_backward_",
             "vae_sample_forward_", "vae_sample_backward_", "sigmoid_backward_", "stn_vae_step_",
             "recon_loss_", "batch_mean_", "clip_adam_", "add_", "rng_fill_",
             "generation_prior_", "asr_pack_", "asr_unpack_", "asr_step_forward_", "asr_terms_",
             "asr_finalize_", "asr_terms_backward_", "asr_step_backward_")
    for n in names:
        getattr(torch.ops.mog_air, n).default  # schema registered
    with pytest.raises(NotImplementedError):
        torch.ops.mog_air.rng_fill_(torch.zeros(4), 1, 0, True)
    # every argument an op writes is annotated as mutated: no
    # schema leaves a written tensor unannotated
    written = {"gemm_f32_": {"C", "Cpre", "colsum"}, "gemm_bf16_": {"C", "colsum"},
               "stn_backward_": {"dU", "dtheta", "dot"},
               "stn_backward_sigmoid_": {"dm", "dtheta", "dot"},
               "lstm_cell_backward_": {"dG", "dc_prev", "dGsum"},
               "lstm_cell_forward2_": {"c_out0", "h_out0", "c_out1", "h_out1"},
               "lstm_cell_backward2_": {"dG0", "dc_prev0", "dGsum0", "dG1", "dc_prev1", "dGsum1"},
               "vae_sample_forward_": {"z", "z_bf16", "runloss", "vkl"},
               "vae_sample_backward_": {"dmu", "dlv", "dmu_bf16", "dlv_bf16"},
               "recon_loss_": {"canvas", "recon", "bce", "mse", "loss", "acc", "dcanvas"},
               "clip_adam_": {"params", "grads", "m", "v", "sumsq"},
               "asr_step_forward_": {"hid", "stop", "digits", "live", "rec"},
               "asr_step_backward_": {"douts", "dpre"}}
    for op, args in written.items():
        sch = getattr(torch.ops.mog_air, op).default._schema
        mut = {a.name for a in sch.arguments if a.alias_info is not None and a.alias_info.is_write}
        assert args <= mut, (op, sorted(args - mut))


def test_functional_ops_registered_and_refuse_cpu():
    """mog_air/torch_ops.py: the differentiable functional ops are registered
    on import and raise on CPU tensors (no CPU implementation)."""
    import mog_air.torch_ops  # noqa: F401
    for n in ("stn", "stn_backward", "lstm_cell", "dense", "glimpse_vae", "stn_vae_step",
              "air_step", "tf_adam_clip_"):
        getattr(torch.ops.mog_air, n).default
    z = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match="HIP device"):
        torch.ops.mog_air.air_step(z, [torch.zeros(8, 2)] * 5, [torch.zeros(2)] * 5,
                                   [torch.zeros(2, 1)] * 5, [torch.zeros(1)] * 5, torch.zeros(4),
                                   torch.zeros(4, 2), torch.zeros(4), torch.zeros(4),
                                   torch.zeros(4), torch.zeros(4, dtype=torch.int32),
                                   torch.ones(1, dtype=torch.int32), [0.0] * 10, True, False)


def test_host_only_entry_point():
    from mog_air import _lib
    assert _lib.load().mog_optim_chunk_elems() == 4096


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from mog_air import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.MogError):
        _lib.load()


def test_param_specs_match_oracle():
    from mog_air.params import param_specs
    cfg = ao.AirConfig()
    mine = param_specs(2500, 256, 784, (512, 256), (256, 512), 50, 64, 64)
    assert mine == ao.param_specs(cfg)
    n = sum(int(np.prod(s)) for _, s in mine)
    assert n == 4011643  # SURVEY.md §0 parameter count


def test_param_store_layout_cpu():
    from mog_air.params import ParamStore, param_specs
    specs = param_specs(2500, 256, 784, (512, 256), (256, 512), 50, 64, 64)
    st = ParamStore(specs, torch.device("cpu"), seed=1)
    for name, shape in specs:
        assert st.offsets[name] % 64 == 0
        assert tuple(st.view(name).shape) == tuple(shape)
    d = st.state_dict()
    st.load_dict({k: v * 0 + 1 for k, v in d.items()})
    assert float(st.flat.sum()) == st.n_params
    assert st.n_blocks == sum(-(-int(np.prod(s)) // 4096) for _, s in specs)


def test_annealing_matches_oracle():
    from mog_air.air_model import annealed_value
    sched = {"init": 10000.0, "min": 1e-9, "factor": 0.1, "iters": 3000,
             "staircase": False, "log": True}
    for step in (0, 1, 100, 3000, 12345, 40000, 10 ** 6):
        assert annealed_value(sched, step) == float(ao.annealed_log_odds(step))


def test_marginal_objective_matches_oracle():
    from mog_air.air_model import marginal_objective
    for prior, T in (((1, 3), 4), ((1, 2, 3), 6), ((2, 4), 6), ((3,), 6)):
        np.testing.assert_array_equal(marginal_objective(prior, T),
                                      ao.marginal_objective(prior, T))


def test_model_rejects_cpu_device():
    from mog_air.air_model import AIRModel
    with pytest.raises(RuntimeError):
        AIRModel(cnn=False, device="cpu")
