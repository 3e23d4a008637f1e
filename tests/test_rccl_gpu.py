"""The DP step's RCCL call sequence executed on a real (one-rank) RCCL communicator.

Multi-rank GPU tests run over gloo (RCCL refuses two ranks on one device); here a subprocess creates
a one-rank NCCL-backend (= RCCL) process group and runs ``utils/rccl_rehearsal.py``: the engine's DP
code path (bucketed async all-reduces between graph segments, the embedding all-gather, the bf16
all-to-all payload chain, ZeRO-1 reduce-scatter / all-gather, the loss all-reduce) with every
collective a one-member identity -- so each configuration must reproduce the same rehearsal run over
gloo bit for bit, and the whole-step capture (``capture_comms``) the cut-graph run."""

import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = [pytest.mark.gpu]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rehearse(backend, cases, td):
    out = os.path.join(td, f"{backend}.pt")
    env = dict(os.environ, DTC_WORLD1_PG="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()))
    env.pop("DTC_DIST_BACKEND", None)
    if backend == "gloo":
        env["DTC_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-u", "-m", "distributed_training_compare_jax_amd.utils.rccl_rehearsal", out,
                        *cases], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return torch.load(out, weights_only=False)


@pytest.fixture(scope="module")
def runs():
    with tempfile.TemporaryDirectory() as td:
        nccl = _rehearse("nccl", ["plain", "fp32", "fp32_captured", "no_gather", "bf16", "bf16_captured", "zero1",
                                  "zero1_captured"], td)
        gloo = _rehearse("gloo", ["fp32", "no_gather", "zero1"], td)
    return nccl, gloo


def test_rccl_primitives_identity(runs):
    nccl, _ = runs
    assert nccl["backend"] == "nccl"
    bad = {k: v for k, v in nccl["primitives"].items() if not v}
    assert not bad, bad


@pytest.mark.parametrize("case", ["fp32", "no_gather", "zero1"])
def test_rccl_dp_path_equals_gloo_bitwise(runs, case):
    nccl, gloo = runs
    a, b = nccl["cases"][case], gloo["cases"][case]
    assert a["dp_comm"] and a["comms"] > 0, a  # the DP path ran, with eager RCCL collectives between segments
    if case == "zero1":
        assert a["zero"]
    assert a["losses"] == b["losses"], (a["losses"], b["losses"])
    assert torch.equal(a["params"], b["params"])


@pytest.mark.parametrize("case", ["fp32", "bf16", "zero1"])
def test_captured_collectives_equal_cut_graphs(runs, case):
    nccl, _ = runs
    cut, cap = nccl["cases"][case], nccl["cases"][case + "_captured"]
    assert cut["graphs"] >= 2 and cut["comms"] > 0
    if case in ("fp32", "zero1"):
        assert cap["graphs"] == 1 and cap["comms"] == 0, cap  # one hipGraph per step, RCCL inside it
    else:  # the bf16 bucket chains stay eager (not capturable); everything else is captured
        assert cap["comms"] < cut["comms"], (cap, cut)
    assert cap["losses"] == cut["losses"]
    assert torch.equal(cap["params"], cut["params"])


def test_rehearsal_tracks_plain_dp1(runs):
    """The rehearsal changes plans (comm-safe GEMMs, 2-layer weight-gradient groups, embedding gather) but
    not the math: it follows the plain dp1 run to bf16 tolerance; the bf16 DP payload adds its rounding."""
    nccl, _ = runs
    ref = nccl["cases"]["plain"]["losses"]
    for case in ("fp32", "bf16"):
        got = nccl["cases"][case]["losses"]
        assert got == pytest.approx(ref, rel=1e-2, abs=1e-2), (case, got, ref)
