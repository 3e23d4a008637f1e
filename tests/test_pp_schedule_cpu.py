"""Pipeline programs (parallel/pp.py) under RCCL point-to-point semantics, without any GPU.

RCCL runs all traffic between two ranks, in issue order, on that pair's communicator stream, and a
send completes only against the matching receive; a buffered backend (gloo, which the CPU layout
tests use) hides ordering bugs that would hang on the real node.  ``pp.simulate`` replays the
static programs of all S stages with per-pair ordered queues, rendezvous matching and grouped calls
as atomic units, and fails on a deadlock or on a message-order mismatch.
"""

import pytest

from distributed_training_compare_jax_amd.parallel import pp as PP


@pytest.mark.parametrize("model", ["pair", "rank"])
@pytest.mark.parametrize("kind", ["gpipe", "1f1b", "zb"])
@pytest.mark.parametrize("S", [1, 2, 3, 4, 8])
def test_programs_never_deadlock(kind, S, model):
    """Both queue models: per-pair streams, and one serialised stream per rank (PyTorch's coalesced
    p2p on RCCL runs every grouped call of a rank on its group communicator's single stream)."""
    for M in range(1, 17):
        c = PP.simulate(kind, S, M, model=model)
        per = 3 if kind == "zb" else 2  # zb: forward, input-gradient backward and weight-gradient items
        assert c["compute"] == per * M * S


@pytest.mark.parametrize("S,M", [(2, 2), (4, 4), (4, 8), (8, 8), (8, 16)])
def test_zero_bubble_programs(S, M):
    """zb = 1F1B's messages in 1F1B's order plus W items: every W after its own B, each microbatch's F, B
    and W exactly once; the timed replay (equal F / B / W costs) shortens the step and the bubble, to at
    most 25 % at 8 stages x 8 microbatches (1F1B: 47 %)."""
    for s, prog in enumerate(PP.zb_programs(S, M)):
        base = PP.pp_program("1f1b", S, s, M)
        assert [it for it in prog if it[0] != "W"] == base  # communication program unchanged
        seen_b = set()
        for it in prog:
            if it[0] == "B":
                seen_b.add(it[1])
            if it[0] == "W":
                assert it[1] in seen_b, (s, it)
        assert sorted(it[1] for it in prog if it[0] == "W") == list(range(M))
    z, o = PP.estimate("zb", S, M), PP.estimate("1f1b", S, M)
    assert z["makespan"] < o["makespan"] and z["bubble"] < o["bubble"]
    if (S, M) == (8, 8):
        assert z["bubble"] <= 0.25, z


@pytest.mark.parametrize("head_split", [False, True])
@pytest.mark.parametrize("S", [2, 3, 4, 8])
def test_zero_bubble_pending_w_bounded(S, head_split):
    """Each pending W keeps its microbatch's dY and X alive: no stage ever holds more than 1F1B's peak
    in-flight count (S, its first stage) of them, also with many microbatches and with a heavy last stage
    (costs that push a stage's W's into the final drain without the cap)."""
    for M in (S, 2 * S, 4 * S, 32):
        costs = PP.stage_item_costs(S, [1.0] * (S - 1) + [3.0])
        for s, prog in enumerate(PP.zb_programs(S, M, costs, head_split=head_split)):
            assert PP.max_pending_w(prog) <= PP.w_cap(S, s), (S, M, s, PP.max_pending_w(prog))
        PP.simulate("zb", S, M, head_split=head_split)  # still deadlock-free under the cap


def test_simulator_catches_the_ungrouped_1f1b_order(monkeypatch):
    """The round-2 executor's order (send, then an ungrouped receive from the same peer) deadlocks
    under blocking semantics as soon as S >= 2 and M >= 2: the simulator must see it."""
    def naive(kind, S, s, M, **kw):
        prog, sends = [], []
        for k, i in PP._schedule(kind, S, s, M):
            if k == "F":
                if s > 0:
                    prog += [("post", f"rf{i}", -1, (), (("f", i),)), ("wait", (f"rf{i}",))]
                prog.append(("F", i))
                if s < S - 1:
                    prog.append(("post", f"sf{i}", +1, (("f", i),), ()))
                    sends.append(f"sf{i}")
            else:
                if s < S - 1:
                    prog += [("post", f"rb{i}", +1, (), (("b", i),)), ("wait", (f"rb{i}",))]
                prog.append(("B", i))
                if s > 0:
                    prog.append(("post", f"sb{i}", -1, (("b", i),), ()))
                    sends.append(f"sb{i}")
        return prog + ([("wait", tuple(sends))] if sends else [])

    monkeypatch.setattr(PP, "pp_program", naive)
    PP.simulate("gpipe", 4, 4)  # GPipe's phases never cross on a pair: fine even ungrouped
    with pytest.raises(RuntimeError, match="deadlock"):
        PP.simulate("1f1b", 2, 2)


@pytest.mark.parametrize("kind", ["gpipe", "1f1b"])
def test_comm_cuts_per_microbatch(kind):
    """Every run of p2p items between two compute items is ONE collective call (one graph cut in a
    replayed step): at most one per compute item + 1, i.e. ~2 per microbatch per stage (round 2:
    recv = post + wait, send = post, each its own cut -> ~6 per microbatch)."""
    S, M = 4, 8
    for s in range(S):
        prog = PP.pp_program(kind, S, s, M)
        runs, prev_comm = 0, False
        for it in prog:
            is_comm = it[0] in ("post", "wait")
            if is_comm and not prev_comm:
                runs += 1
            prev_comm = is_comm
        assert runs <= 2 * M + 1, (s, runs)


def test_rank_model_is_stricter(monkeypatch):
    """A three-rank send cycle whose receives sit second on each rank: fine with per-pair streams, a
    deadlock once each rank's posts serialise on one stream (the rank model must see it)."""
    progs = {
        0: [("post", "a", +1, (("f", 0),), ()), ("post", "c", +2, (), (("x", 0),)), ("wait", ("a", "c"))],
        1: [("post", "b", +1, (("f", 1),), ()), ("post", "a", -1, (), (("f", 0),)), ("wait", ("a", "b"))],
        2: [("post", "c", -2, (("x", 0),), ()), ("post", "b", -1, (), (("f", 1),)), ("wait", ("b", "c"))],
    }
    monkeypatch.setattr(PP, "pp_program", lambda kind, S, s, M: progs[s])
    PP.simulate("gpipe", 3, 1, model="pair")
    with pytest.raises(RuntimeError, match="deadlock"):
        PP.simulate("gpipe", 3, 1, model="rank")


@pytest.mark.parametrize("kind", ["1f1b", "zb"])
@pytest.mark.parametrize("S", [2, 3, 4, 8])
@pytest.mark.parametrize("M", [1, 2, 3, 8, 16])
def test_head_split_programs_are_deadlock_free(kind, S, M):
    """pp_head_split: the last two stages' extra row-statistics exchange (H / exchange / Hf) keeps the
    programs deadlock-free and matched under both queue models; every stage still runs each F, B once and
    the two head stages one H and one Hf per microbatch."""
    for model in ("pair", "rank"):
        PP.simulate(kind, S, M, model=model, head_split=True)
    progs = PP.zb_programs(S, M, head_split=True) if kind == "zb" else \
        [PP.pp_program(kind, S, s, M, head_split=True) for s in range(S)]
    for s, prog in enumerate(progs):
        kinds = [it[0] for it in prog if it[0] in ("F", "B", "H", "Hf")]
        assert kinds.count("B") == M
        assert kinds.count("H") == kinds.count("Hf") == (M if s >= S - 2 else 0)
        assert kinds.count("F") == (0 if s == S - 1 else M)


def test_head_split_estimate_gpt2_small_pp8():
    """GPT-2 small at pp8 (M 8): the head alone (2.9 blocks) bounds the unsplit pipeline; halving it over the
    last two stages cuts the predicted step by > 15 % under 1F1B and zero-bubble alike."""
    from distributed_training_compare_jax_amd.parallel.mesh import split_layers, stage_costs

    hc = 2.89
    res = {}
    for hs in (1, 2):
        r = split_layers(12, 8, (0.05, hc), head_stages=hs)
        c = PP.stage_item_costs(8, stage_costs(r, (0.05, hc), hs), head_half=hc / 2 if hs == 2 else 0.0)
        for kind in ("1f1b", "zb"):
            res[(hs, kind)] = PP.estimate(kind, 8, 8, c, head_split=hs == 2)
    assert [len(x) for x in split_layers(12, 8, (0.05, hc), head_stages=2)] == [2, 2, 2, 2, 2, 2, 0, 0]
    for kind in ("1f1b", "zb"):
        assert res[(2, kind)]["makespan"] < 0.85 * res[(1, kind)]["makespan"], (kind, res)
    assert res[(2, "zb")]["bubble"] < res[(1, "zb")]["bubble"]
