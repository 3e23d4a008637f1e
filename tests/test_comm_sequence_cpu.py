"""Cross-rank collective-sequence check (parallel/program.py): every group's members must issue the
same collectives in the same order, and every send must meet its receive — the property whose
violation is a silent RCCL hang.  The checker itself, then the real StepProgram over gloo with
2 ranks: agreeing ranks pass, a rank-dependent extra collective or a shape mismatch raises on
every rank (instead of hanging).  Real DP / TP / PP / hybrid steps run the same check on their first
step (Engine.run_step), so every multi-rank case of test_parallel_cpu.py also exercises it."""

import os
import tempfile

import pytest
import torch

from distributed_training_compare_jax_amd.parallel.dist import spawn
from distributed_training_compare_jax_amd.parallel.program import check_collective_sequences


def _c(op, ranks, *shapes):
    return ("coll", op, tuple(ranks), tuple((tuple(s), "float32") for s in shapes))


def test_checker_accepts_matching_sequences():
    a = [_c("all_reduce", (0, 1), (8,)), _c("all_reduce", (0, 2), (4,))]
    b = [_c("all_reduce", (0, 1), (8,)), ("send", 3, ((2, 2), "float32"))]
    c = [_c("all_reduce", (0, 2), (4,))]
    d = [("recv", 1, ((2, 2), "float32"))]
    assert check_collective_sequences([a, b, c, d]) is None


def test_checker_names_first_disagreement():
    a = [_c("all_reduce", (0, 1), (8,)), _c("all_reduce", (0, 1), (1,))]
    b = [_c("all_reduce", (0, 1), (8,)), _c("all_gather", (0, 1), (1,))]
    err = check_collective_sequences([a, b])
    assert err is not None and "collective #1" in err and "all_gather" in err
    # a missing collective on one member
    err = check_collective_sequences([a, a[:1]])
    assert err is not None and "nothing" in err
    # a collective on a group the rank is not in
    err = check_collective_sequences([[_c("all_reduce", (1, 2), (1,))], [], []])
    assert err is not None and "not a member" in err


def test_checker_pairs_sends_with_receives_in_order():
    x, y = ((4, 8), "bfloat16"), ((4, 8), "float32")
    ok = [[("send", 1, x), ("send", 1, y)], [("recv", 0, x), ("recv", 0, y)]]
    assert check_collective_sequences(ok) is None
    swapped = [[("send", 1, x), ("send", 1, y)], [("recv", 0, y), ("recv", 0, x)]]
    err = check_collective_sequences(swapped)
    assert err is not None and "p2p 0 -> 1" in err and "#0" in err
    unmatched = [[("send", 1, x)], []]
    assert "1 sends, 0 receives" in check_collective_sequences(unmatched)


def _prog_worker(case, out_dir):
    import torch.distributed as dist

    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.parallel.program import StepProgram, csig

    d = init_distributed("cpu")
    p = StepProgram(torch.device("cpu"), use_graph=False)
    t = torch.ones(8 if (case == "shape" and d.rank == 1) else 4)
    g = dist.group.WORLD
    p.collect()
    if case == "shape":
        # same op, different message size on rank 1: only the signature is issued (the real call would hang)
        p.comm(lambda: None, sig=csig("all_reduce", g, t))
    else:
        p.comm(lambda: dist.all_reduce(t), sig=csig("all_reduce", g, t))
    if case == "extra" and d.rank == 1:
        # a rank-dependent collective: only the signature is recorded (running it would hang rank 0)
        p.comm(lambda: None, sig=csig("all_reduce", g, t))
    err = ""
    try:
        p.verify("test step")
    except RuntimeError as e:
        err = str(e)
    torch.save(err, os.path.join(out_dir, f"r{d.rank}.pt"))
    destroy()


@pytest.mark.parametrize("case", ["ok", "extra", "shape"])
def test_step_program_verify_two_ranks(case):
    with tempfile.TemporaryDirectory() as td:
        spawn(_prog_worker, 2, args=(case, td))
        errs = [torch.load(os.path.join(td, f"r{r}.pt")) for r in range(2)]
    if case == "ok":
        assert errs == ["", ""]
    else:
        # every rank raises the same diagnosis
        assert errs[0] and errs[0] == errs[1], errs
        assert "ranks disagree on the collectives of the test step" in errs[0]
        assert ("(1 vs 2 collectives per step)" in errs[0]) if case == "extra" else ("(4,)" in errs[0] and "(8,)" in errs[0])
