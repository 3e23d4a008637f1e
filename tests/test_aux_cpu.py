"""Auxiliary subsystems on CPU: watchdog (failure detection) and step tracing."""

import json
import os
import time

import torch

from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
from distributed_training_compare_jax_amd.parallel.dist import DistInfo
from distributed_training_compare_jax_amd.train.loop import train
from distributed_training_compare_jax_amd.utils.watchdog import Watchdog


def test_watchdog_fires_on_stall(capfd):
    codes = []
    dog = Watchdog(rank=3, timeout_s=0.2, exit_fn=codes.append).start()
    dog.beat(7)
    time.sleep(0.8)
    dog.stop()
    assert codes == [124] and dog.fired
    err = capfd.readouterr().err
    assert "[rank 3] watchdog" in err and "last completed step 7" in err


def test_watchdog_quiet_while_beating():
    codes = []
    with Watchdog(rank=0, timeout_s=0.3, exit_fn=codes.append) as dog:
        for i in range(8):
            dog.beat(i)
            time.sleep(0.05)
    assert codes == [] and not dog.fired


def test_profile_writes_trace_and_metrics(tmp_path):
    mc = model_config_from_preset("tiny", vocab_size=500)
    tc = TrainConfig(seed=0, parallel="dp", batch=2, steps=3, log_every=100, output_dir=str(tmp_path), device="cpu",
                     warmup_steps=1, profile=True)
    r = train(tc, mc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), DistInfo(0, 1, 0, torch.device("cpu"), "gloo"), quiet=True)
    tr = json.load(open(os.path.join(tmp_path, "trace", "rank0.json")))
    names = {e["name"] for e in tr["traceEvents"]}
    assert {"data", "loss sync", "step 1", "step 3"} <= names
    m = json.load(open(os.path.join(tmp_path, "metrics.json")))
    assert m["trace"].endswith("rank0.json")


def test_native_data_sampler_matches_numpy():
    """The C++ sampler (csrc/host_data.cpp -> _dtc_host.so) yields the numpy stream bit for bit,
    at offsets/lengths crossing row boundaries, both vocabularies and a position past 2^40."""
    import numpy as np

    from distributed_training_compare_jax_amd.csrc.build import build_host
    from distributed_training_compare_jax_amd.data import synthetic as S

    build_host()
    S._host = None  # re-probe now that the library exists
    for vocab, seed in ((S.BPE_VOCAB, 0), (999, 7)):
        s = S.SyntheticTokenStream(vocab=vocab, seed=seed, native=True)
        for start, count in ((0, 1), (0, 4104), (1, 513), (98765, 20000), (1 << 41, 3000)):
            a, b = s.tokens(start, count), s.tokens_numpy(start, count)
            assert a.dtype == np.int32 and np.array_equal(a, b), (vocab, seed, start, count)
    # the iterator (what bench.py / main.py consume) is unchanged by the native path
    it_n = S.get_batch_iterator(4, 513, seed=1, row0=1, nrows=2)
    ref = S.SyntheticTokenStream(seed=1, native=False)
    for step in range(3):
        assert np.array_equal(next(it_n), ref.rows(step, 1, 2, 4, 513))
