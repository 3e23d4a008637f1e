"""DP gradient buckets (parallel/dp.py): layer-aligned cuts and issue points."""

import torch

from distributed_training_compare_jax_amd.config.schema import ModelConfig
from distributed_training_compare_jax_amd.models.params import stage_param_specs
from distributed_training_compare_jax_amd.parallel.buffers import FlatParams
from distributed_training_compare_jax_amd.parallel.dp import GradBuckets


class _Prog:
    def __init__(self):
        self.issued = []

    def comm(self, fn, name=None, sig=None):
        self.issued.append(name)


def _ref_flat():
    mc = ModelConfig(vocab_size=50258, d_model=512, n_layers=12, n_heads=16, d_ff=2048, max_seq_len=512, dropout=0.1)
    return FlatParams(stage_param_specs(mc, range(12), True, True), 0, 1, "cpu", compute_dtype=torch.float32)


def _bounds(f, layers):
    names = list(f.slots)
    ends = [f.range_of([n for n in names if n.startswith(f"h.{l}.")])[1] for l in layers]
    head = f.range_of([n for n in names if n.startswith("lm_head") or n.startswith("lnf")])[1]
    return ends, head


def test_layer_aligned_buckets_reference_model():
    f = _ref_flat()
    ends, head = _bounds(f, range(12))
    prog = _Prog()
    b = GradBuckets(f, None, 8, prog, 40.0, 16.0, local_names=("wte", "wpe"), boundaries=ends + [head])
    mb = [round((c - a) * 4 / 2 ** 20, 1) for a, c in b.buckets]
    assert mb == [98.4, 48.1, 48.1, 36.1, 12.0]
    # buckets tile [0, reduce_end) and every cut is a layer / head boundary
    assert b.buckets[0][0] == 0 and b.buckets[-1][1] == b.reduce_end
    assert all(x[1] == y[0] for x, y in zip(b.buckets, b.buckets[1:]))
    assert all(c in set(ends + [head]) for _, c in b.buckets)
    # issue points: the head bucket right after the head backward, then a bucket as soon as its
    # last layer (backward order 11 -> 0) is done; the tail (layer 0) only at the end
    b.ready_upto(b.head_end_offset())
    assert prog.issued == ["dp_bucket0"]
    seen = {}
    for l in reversed(range(12)):
        b.ready_upto(b.layer_end_offset(l))
        seen[l] = list(prog.issued)
    assert seen[8][-1] == "dp_bucket1" and seen[4][-1] == "dp_bucket2" and seen[1][-1] == "dp_bucket3"
    assert seen[0][-1] == "dp_bucket4" and len(prog.issued) == 5


def test_param_cut_buckets_unchanged_without_boundaries():
    f = _ref_flat()
    b = GradBuckets(f, None, 8, _Prog(), 64.0, 16.0, local_names=("wte", "wpe"))
    assert b.buckets[0][0] == 0 and b.buckets[-1][1] == b.reduce_end
    assert sum(c - a for a, c in b.buckets) == b.reduce_end


def test_bf16_payload_chain_is_never_captured():
    """The bf16 payload chain issues its collectives from a side stream forked into the step; an RCCL
    collective issued from a stream forked into a hipGraph capture segfaults at capture end (root cause:
    benchmarks/capture_side_stream_probe.py, docs/CAPTURE.md), so the chain must always be registered as
    a non-capturable (eager, graph-cutting) item -- and the fp32 all-reduce buckets as capturable."""
    class Prog:
        def __init__(self):
            self.cap = {}

        def comm(self, fn, name=None, sig=None, capturable=True):
            self.cap[name] = capturable

    f = _ref_flat()
    ends, head = _bounds(f, range(12))
    for payload, want in (("bf16", False), ("fp32", True)):
        prog = Prog()
        b = GradBuckets(f, None, 8, prog, 40.0, 16.0, local_names=("wte", "wpe"), boundaries=ends + [head],
                        payload=payload)
        b.ready_all()
        assert len(prog.cap) == len(b.buckets) and all(v is want for v in prog.cap.values()), (payload, prog.cap)
