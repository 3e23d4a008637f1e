"""Scheduling logic of the batched gradient reducer (ops/reduce.py) on CPU: which tasks each
flush launches, the one-flush lag of grad-norm tasks behind the reductions that produce their
inputs, block ordering inside a launch and batch splitting (the device kernel itself is tested on
the GPU: tests/test_kernels_gpu.py::test_batched_reducer_matches_per_op)."""

import torch

from distributed_training_compare_jax_amd.ops import reduce as R


class Recorder(R.GradReducer):
    def __init__(self):
        super().__init__("cpu")
        self.batches = []

    def _launch(self, tasks):
        for i in range(0, len(tasks), R.MAX_TASKS):
            self.batches.append([t[0] for t in tasks[i:i + R.MAX_TASKS]])


def test_sumsq_waits_for_the_flush_that_finalizes_its_grads():
    r = Recorder()
    dst, data, part = torch.zeros(8), torch.zeros(16), torch.zeros(2)
    # layer L: reductions queued, flushed; its norm chunk is queued after the flush
    r.add_wide(torch.zeros(2, 8), dst, 2, 0.0)
    r.add_tall(0, 8, 4, dst, 0.0)
    r.flush()
    assert r.batches == [[R.RED_TALL, R.RED_WIDE]]  # TALL blocks dispatched first
    r.add_sumsq(data, 1.0, part)
    # layer L-1: its reductions + layer L's norm chunk go out together (norm blocks first)
    r.add_wide(torch.zeros(2, 8), dst, 2, 0.0)
    r.flush()
    assert r.batches[-1] == [R.RED_SUMSQ, R.RED_WIDE]
    assert not r.sumsq and not r.pending


def test_sumsq_added_with_pending_reductions_waits_one_more_flush():
    r = Recorder()
    dst, data, part = torch.zeros(8), torch.zeros(16), torch.zeros(2)
    r.add_wide(torch.zeros(2, 8), dst, 2, 0.0)
    r.add_sumsq(data, 1.0, part)  # its inputs may be written by the pending reduction
    r.flush()
    assert r.batches == [[R.RED_WIDE]]
    r.flush_all()
    assert r.batches[-1] == [R.RED_SUMSQ]


def test_flush_all_drains_and_batches_split():
    r = Recorder()
    dst = torch.zeros(8)
    for _ in range(R.MAX_TASKS + 3):
        r.add_tall(0, 8, 4, dst, 1.0)
    r.flush_all()
    assert [len(b) for b in r.batches] == [R.MAX_TASKS, 3]
    r.flush()  # nothing queued: no launch
    assert len(r.batches) == 2


def test_arena_window_resets_on_flush():
    r = Recorder()
    r.arena_bytes = 1 << 16
    a = r.alloc(100)
    b = r.alloc(100)
    assert b.data_ptr() - a.data_ptr() == 512  # 256-B granules
    r.flush()
    c = r.alloc(100)
    assert c.data_ptr() == a.data_ptr()
