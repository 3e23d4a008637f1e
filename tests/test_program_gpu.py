"""StepProgram capture: graph segments that captured nothing (two collectives back to back, a collective
then its wait) are dropped instead of replayed as empty hipGraphs; the program still replays the kept
segments and the collectives in their recorded order."""

import pytest
import torch

from distributed_training_compare_jax_amd.parallel.program import StepProgram

pytestmark = pytest.mark.gpu


def test_program_drops_empty_segments(cuda):
    prog = StepProgram(cuda, use_graph=True)
    x = torch.zeros(4, device=cuda)
    order = []

    def step():
        x.add_(1)
        prog.comm(lambda: order.append(("comm", float(x[0]))), name="a")
        prog.wait("a")  # nothing captured between the collective and its wait
        prog.comm(lambda: order.append(("comm2", float(x[0]))))
        x.mul_(3)

    prog.record(step)
    assert prog.n_graphs == 2 and prog.n_comms == 3, prog.items
    assert len(prog._empty) == 2
    kinds = [k for k, _, _ in prog.items]
    assert kinds == ["graph", "comm", "wait", "comm", "graph"]
    for _ in range(2):
        prog.replay()
    torch.cuda.synchronize()
    # replay 1: x = (0 + 1) * 3 = 3; replay 2: (3 + 1) * 3 = 12; each comm sees the value after the add
    assert torch.equal(x, torch.full((4,), 12.0, device=cuda))
    assert order == [("comm", 1.0), ("comm2", 1.0), ("comm", 4.0), ("comm2", 4.0)]
