"""Device-side bounds checks: the step's kernels built with ``-DDTC_DEBUG`` (every ``DTC_ASSERT`` of
their index math live, ``csrc/build.py --debug`` -> ``_dtc_kernels_debug.so``) run GPT-2-small-shaped
training steps (d768, T1024, hd64, vocab 50258, batch 8 = 8192 tokens: the headline step's kernel
plans; 2 layers to keep the -O1 build quick) and must match the release library's losses.

Each library runs in its own subprocess (``DTC_KERNEL_LIB`` selects it at load), so a failed device
assert aborts that child only and the test reports which library and what it printed."""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_training_compare_jax_amd")

SCRIPT = r"""
import torch
from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
from distributed_training_compare_jax_amd.data.synthetic import get_batch_iterator
from distributed_training_compare_jax_amd.parallel.dist import DistInfo
from distributed_training_compare_jax_amd.train.engine import Engine
from distributed_training_compare_jax_amd.ops import _native as N

dev = torch.device("cuda:0")
mc = model_config_from_preset("gpt2-small", vocab_size=50258, n_layers=2)
tc = TrainConfig(seed=0, parallel="dp", batch=8, steps=3, log_every=1, output_dir="/tmp/x", use_graph=True)
oc = OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0)
eng = Engine(mc, tc, oc, DistInfo(0, 1, 0, dev, "nccl"))
it = get_batch_iterator(8, mc.max_seq_len + 1)
losses = []
for _ in range(3):
    eng.set_batch(next(it))
    eng.run_step()
    losses.append(eng.loss_value())
torch.cuda.synchronize()
print("LIB", N.LIB_PATH)
print("LOSSES", " ".join(f"{x:.6f}" for x in losses))
"""


def _run(lib):
    env = dict(os.environ, DTC_KERNEL_LIB=lib, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"{os.path.basename(lib)} exited {r.returncode}:\n{out[-4000:]}"
    libs = [l for l in r.stdout.splitlines() if l.startswith("LIB ")]
    assert libs and libs[0].split()[1] == lib, out[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("LOSSES ")]
    assert line, out[-4000:]
    return [float(x) for x in line[0].split()[1:]]


def test_debug_kernels_assert_clean_and_match_release():
    dbg = os.path.join(PKG, "_dtc_kernels_debug.so")
    rel = os.path.join(PKG, "_dtc_kernels.so")
    assert os.path.exists(dbg), "debug kernel library missing: __graft_entry__.build() builds it in-tree"
    ld = _run(dbg)
    lr = _run(rel)
    for a, b in zip(ld, lr):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), (ld, lr)
