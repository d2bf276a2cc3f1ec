"""End-to-end runs of the kept entry point (training_air_original.py) on the
GPU: offline synthetic data, a few train iterations, the final test-model
evaluation and its log lines (training_air_original.py:412-503)."""
import glob
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("data,precision", [("mnist", "fp32"), ("dsprites", "bf16")])
def test_training_air_original_runs(tmp_path, monkeypatch, data, precision):
    import training_air_original as entry
    monkeypatch.chdir(tmp_path)  # results/ and data/ paths are relative, as in the reference
    step = entry.main(["-dn", "13" if data == "mnist" else "24", "-data", data, "-r",
                       str(tmp_path / "res"), "-k", "t", "--iterations", "21",
                       "--synth-per-count", "40", "--precision", precision])
    assert step == 21
    logs = glob.glob(str(tmp_path / "res_(t)" / "logfile*.log"))
    assert logs
    text = open(logs[0]).read()
    assert "iteration 20\ttrain loss" in text
    assert "iteration final\ttest loss" in text and "globaliou" in text
    assert "training has ended" in text
    assert glob.glob(str(tmp_path / "res_(t)" / "models" / "air-model-0.npz"))
