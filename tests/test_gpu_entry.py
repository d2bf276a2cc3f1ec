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


@pytest.mark.parametrize("flags", [["-dn", "13", "-gm", "100", "-gne", "10"],
                                   ["-dn", "3", "-ds", "bbox", "-gb", "1", "-ga", "0.1",
                                    "--precision", "bf16"]])
def test_train_air_pr_runs(tmp_path, monkeypatch, flags):
    import train_air_pr as entry
    monkeypatch.chdir(tmp_path)
    step = entry.main(flags + ["-r", str(tmp_path / "res"), "-k", "p", "--iterations", "21",
                               "--synth-per-count", "40"])
    assert step == 21
    text = open(glob.glob(str(tmp_path / "res_(p)" / "logfile*.log"))[0]).read()
    assert "step:    20\t" in text and "num_margin" in text and "TotLoss" in text
    # the ASR trainer logs its final test under the step number
    # (train_air_pr.py:426-430), unlike training_air_original.py's 'final'
    assert "test:    21\tprecision" in text and "training has ended" in text
