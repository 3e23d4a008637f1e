"""End-to-end: ``main.py`` with each reference train YAML (tiny model, CPU/gloo), checking the
console contract (reference train/train.py prints) and the ``log.csv`` schema."""

import os
import re
import shutil
import subprocess
import sys

import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, train_yaml, nproc=1, steps=4):
    shutil.copytree(os.path.join(ROOT, "configs"), tmp_path / "configs")
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "main.py"), "--train_config_path", f"configs/{train_yaml}",
           "--model_config_path", "configs/model_config_tiny.yaml", "--steps", str(steps), "--device", "cpu",
           "--log_every", "2", "--warmup_steps", "2", "--nproc", str(nproc)]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.slow
@pytest.mark.parametrize("yaml,strategy,nproc", [("train_config_dp.yaml", "dp", 1), ("train_config_tp.yaml", "tp", 2),
                                                 ("train_config_pp.yaml", "pp", 2)])
def test_main_cli(tmp_path, yaml, strategy, nproc):
    out = _run(tmp_path, yaml, nproc)
    lines = [l for l in out.strip().splitlines() if not l.startswith("[Gloo]")]  # gloo library chatter
    assert lines[0] == f"Running `{strategy}` on {nproc} devices."
    assert "Warmup" in lines and "Start measuring" in lines and lines[-1] == "End"
    steps = [l for l in lines if l.startswith("Step:")]
    assert len(steps) == 2
    assert re.fullmatch(r"Step: 2 \| Avg loss: \d+\.\d{4} \| Average step time: \d+\.\d{4}", steps[0])
    assert any(l.startswith("Total time: ") for l in lines)
    df = pd.read_csv(tmp_path / "outputs" / strategy / "log.csv")
    assert list(df.columns) == ["step", "elapsed_time", "loss"]
    assert df.step.tolist() == [0, 1, 2, 3]
    assert (df.elapsed_time.diff().dropna() > 0).all()
    assert df.loss.between(5, 12).all()


@pytest.mark.slow
def test_main_cli_zero1(tmp_path):
    """configs/train_config_dp_zero1.yaml: DP with ZeRO-1 optimizer-state sharding over 2 ranks."""
    out = _run(tmp_path, "train_config_dp_zero1.yaml", nproc=2)
    assert "Running `dp` on 2 devices." in out
    df = pd.read_csv(tmp_path / "outputs" / "dp_zero1" / "log.csv")
    assert df.step.tolist() == [0, 1, 2, 3] and df.loss.between(5, 12).all()


def test_unknown_strategy_rejected(tmp_path):
    shutil.copytree(os.path.join(ROOT, "configs"), tmp_path / "configs")
    (tmp_path / "configs" / "bad.yaml").write_text(
        "batch: 8\nlog_every: 1\noutput_dir: x\nparallel: zz\nseed: 0\nsteps: 1\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--train_config_path", "configs/bad.yaml",
                        "--device", "cpu", "--nproc", "1"], cwd=tmp_path, env=dict(os.environ, PYTHONPATH=ROOT),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "Unsupported strategy `zz`" in r.stderr
