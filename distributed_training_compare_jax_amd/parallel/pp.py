"""Pipeline-parallel schedules over RCCL point-to-point send/recv.

Reference PP (``train/create_train_step.py:55-195``): GPipe fill/drain expressed as a
``lax.scan`` over ``M+S-1`` clocks where EVERY stage runs ``lax.cond``-gated work on every
clock and ``ppermute`` shifts activations, labels and a valid flag each clock (also on
bubble clocks); backward is autodiff of the scan.  Here each stage runs a host-side static
PROGRAM (:func:`pp_program`) of compute items and communication entries:

* only valid (stage, microbatch) work exists — no bubble-clock compute or traffic;
* labels never travel (every rank reads its own rows; reference ppermutes them, ``:165``);
* activations travel as fp32 ``[mb·T, D]`` (the residual stream), gradients likewise;
* ``gpipe`` = reference order (all forwards, then all backwards) with the receive of the next
  microbatch posted BEFORE the current one computes (the transfer runs under the compute);
* ``1f1b`` = PipeDream-flush order (activation memory bounded by S microbatches instead of M), with
  Megatron's paired exchanges: in the steady state the send of a forward output and the receive of
  a backward gradient — both with the next stage — are ONE grouped RCCL call
  (``batch_isend_irecv``), and likewise send-gradient/receive-activation with the previous stage.
* ``zb`` = zero-bubble-style 1F1B (Qi et al., "Zero Bubble Pipeline Parallelism", ZB-H1 memory): the
  backward splits into B (the input-gradient chain: every dgrad GEMM, attention and LayerNorm backward
  -- what the previous stage waits for) and W (the stage's deferred weight gradients, one grouped launch,
  ``models/gpt.py`` wgrad queue).  The communication program is exactly 1F1B's (so its deadlock freedom
  carries over); W items carry no messages and are placed by :func:`zb_program` where a timed replay of
  the pipeline (:func:`timeline`, per-item costs) shows the stage idle waiting for a message -- the
  cool-down bubble fills with weight gradients instead of idle time.

Why the pairing matters on RCCL: all p2p traffic between two ranks runs, in issue order, on that
pair's communicator stream, and a send completes only against the matching receive.  Two stages
that each issue "send to you" before "receive from you" therefore wait on each other forever (a
buffered backend such as gloo hides this).  A grouped call is one kernel that makes progress on
both directions at once.  :func:`simulate` replays the programs of all stages under exactly these
semantics (per-pair ordered queues, rendezvous matching, groups atomic) and is run by the CPU tests
for every S / M / schedule the engine accepts — no-deadlock and message order by construction.

Loss/gradient scaling is exact: each microbatch's CE is scaled by ``1/(mb·T·M)`` so the
sum over microbatches is the full-batch mean (reference: ``psum(loss_sum / M)``, ``:187``).
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from ..ops.optim import cast_to_bf16, fill_
from ..ops.payload import cast_bf16_to_f32
from .dist import staged_p2p
from .program import psig

# ------------------------------------------------------------------------------ static programs
# items: ("F", i) / ("B", i) / ("W", i)              compute of microbatch i (W: zb only)
#        ("H", i) / ("Hf", i)                         head split only: this stage's vocab half of lm_head + CE
#                                                    (logits + row statistics) / the loss from both halves
#        ("post", name, peer, sends, recvs)          one (grouped) p2p call with stage s+peer;
#                                                    sends/recvs: tuples of tags ("f"|"b"|"s", i)
#        ("wait", names)                              the compute stream waits for these entries
# tag ("f", i): activation of microbatch i, stage s -> s+1; ("b", i): its gradient, s+1 -> s; ("s", i): the
# head split's row statistics, exchanged both ways between the last two stages.


def _schedule(kind: str, S: int, s: int, M: int) -> List[tuple]:
    """Compute order ('F', mb) / ('B', mb) for stage s of S."""
    if kind == "gpipe" or S == 1:
        return [("F", i) for i in range(M)] + [("B", i) for i in reversed(range(M))]
    if kind != "1f1b":
        raise ValueError(f"unknown pp_schedule {kind}")
    warm = min(S - s - 1, M)
    ops = [("F", i) for i in range(warm)]
    f, b = warm, 0
    while f < M:
        ops.append(("F", f))
        f += 1
        ops.append(("B", b))
        b += 1
    while b < M:
        ops.append(("B", b))
        b += 1
    return ops


def _head_split(prog: List[tuple], S: int, s: int) -> List[tuple]:
    """``pp_head_split``: lm_head + CE by vocab halves on the last two stages A = S-2 and B = S-1.  A's F
    ends with the final LayerNorm, whose output is the f message to B; right after sending it (and after
    the wait its grouped call carries) A computes its half (H), exchanges the row statistics with B (one
    grouped send + receive) and finalises the loss (Hf).  B's F is just H, exchange, Hf; B's backward sends
    its half's input-gradient partial as the usual b message, which A adds before the LayerNorm backward.
    Both stages post the exchange of microbatch i after the f message of i on their pair queue, so the
    1F1B pairing and its deadlock freedom carry over (:func:`simulate` checks every S, M)."""
    def exch(i, peer):
        return [("H", i), ("post", f"s{i}", peer, (("s", i),), (("s", i),)), ("wait", (f"s{i}",)), ("Hf", i)]

    if s == S - 1:
        out = []
        for it in prog:
            out += exch(it[1], -1) if it[0] == "F" else [it]
        return out
    if s != S - 2:
        return prog
    out: List[tuple] = []
    pending = None  # microbatch whose f message was just posted
    for k, it in enumerate(prog):
        out.append(it)
        if it[0] == "post" and any(t[0] == "f" for t in it[3]) and it[2] > 0:
            pending = [t[1] for t in it[3] if t[0] == "f"][0]
            nxt = prog[k + 1] if k + 1 < len(prog) else None
            if not (nxt and nxt[0] == "wait" and it[1] in nxt[1]):
                out += exch(pending, +1)
                pending = None
        elif it[0] == "wait" and pending is not None:
            out += exch(pending, +1)
            pending = None
    return out


def pp_program(kind: str, S: int, s: int, M: int, costs=None, head_split: bool = False, comm=0.0) -> List[tuple]:
    if kind == "zb":
        return zb_programs(S, M, costs, comm, head_split=head_split)[s]
    if head_split:
        if kind != "1f1b" or S < 2:
            raise ValueError("pp_head_split needs pp >= 2 and the 1f1b or zb schedule")
        return _head_split(pp_program(kind, S, s, M), S, s)
    first, last = s == 0, s == S - 1
    prog: List[tuple] = []
    sends: List[str] = []

    def post(name, peer, snd=(), rcv=()):
        prog.append(("post", name, peer, tuple(snd), tuple(rcv)))
        return name

    def send_f(i):
        if not last:
            sends.append(post(f"sf{i}", +1, snd=[("f", i)]))

    def send_b(i):
        if not first:
            sends.append(post(f"sb{i}", -1, snd=[("b", i)]))

    if kind == "gpipe" or S == 1:
        # all forwards, then all backwards (reverse microbatch order); the receive of the next
        # microbatch of the same phase is posted before the current one computes
        for phase in ("F", "B"):
            mbs = list(range(M)) if phase == "F" else list(reversed(range(M)))
            has = (not first) if phase == "F" else (not last)
            d, peer = ("f", -1) if phase == "F" else ("b", +1)
            if has:
                post(f"r{d}{mbs[0]}", peer, rcv=[(d, mbs[0])])
            for n, i in enumerate(mbs):
                if has:
                    prog.append(("wait", (f"r{d}{i}",)))
                    if n + 1 < len(mbs):
                        post(f"r{d}{mbs[n + 1]}", peer, rcv=[(d, mbs[n + 1])])
                prog.append((phase, i))
                send_f(i) if phase == "F" else send_b(i)
        if sends:
            prog.append(("wait", tuple(sends)))
        return prog

    if kind != "1f1b":
        raise ValueError(f"unknown pp_schedule {kind}")
    warm = min(S - s - 1, M)

    def recv_f(i):
        if not first:
            prog.append(("wait", (post(f"rf{i}", -1, rcv=[("f", i)]),)))

    def recv_b(i):
        if not last:
            prog.append(("wait", (post(f"rb{i}", +1, rcv=[("b", i)]),)))

    for i in range(warm):
        recv_f(i)
        prog.append(("F", i))
        send_f(i)
    rem = M - warm
    if rem > 0:
        recv_f(warm)
    for j in range(rem):
        i = warm + j
        prog.append(("F", i))
        if not last:  # send_forward + recv_backward with the next stage: one grouped call
            n = post(f"xf{i}b{j}", +1, snd=[("f", i)], rcv=[("b", j)])
            prog.append(("wait", (n,)))
        prog.append(("B", j))
        if j == rem - 1:
            send_b(j)
        elif not first:  # send_backward + recv_forward with the previous stage
            n = post(f"xb{j}f{i + 1}", -1, snd=[("b", j)], rcv=[("f", i + 1)])
            prog.append(("wait", (n,)))
    for j in range(rem, M):
        recv_b(j)
        prog.append(("B", j))
        send_b(j)
    if sends:
        prog.append(("wait", tuple(sends)))
    return prog


# ------------------------------------------------------------------------------ zero bubble (B/W split)
def stage_item_costs(S: int, stage_cost=None, split=(1.0, 1.0, 1.0), head_half: float = 0.0) -> List[Dict[str, float]]:
    """Per-stage cost of one microbatch's F, B (input-gradient chain) and W (weight gradients), in any
    unit.  ``stage_cost[s]``: the stage's relative size (``mesh.stage_costs``: its layers + the head's
    block-equivalents on the last stage); ``split``: the F : B : W ratio of a block (a block's backward is
    ~2x its forward, half of it the dgrads, half the weight gradients)."""
    stage_cost = [1.0] * S if stage_cost is None else list(stage_cost)
    tot = float(sum(split))
    out = [dict({k: c * v / tot for k, v in zip("FBW", split)}, H=0.0, Hf=0.0) for c in stage_cost]
    if head_half > 0 and S >= 2:  # pp_head_split: the head half's forward is the H item of the last two stages
        for c in out[-2:]:
            h = head_half * split[0] / tot
            c["H"] = h
            c["F"] = max(0.0, c["F"] - h)
    return out


def _comm_cost(comm, tags) -> float:
    """Transfer time of one (grouped) entry: ``comm`` a number (every message), or a dict by tag kind
    ({"f": .., "b": .., "s": ..}: activations / gradients / the head split's row statistics) -- the largest
    message of the group."""
    if not isinstance(comm, dict):
        return float(comm)
    return max((float(comm.get(t[0], 0.0)) for t in tags), default=0.0)


def timeline(progs: List[List[tuple]], costs: List[Dict[str, float]], comm: float = 0.0,
             model: str = "rank") -> Dict[str, object]:
    """Timed replay of the stages' programs: every stage runs its items in order on one clock (compute
    items take ``costs[s][kind]``, a post records its time, a wait advances the clock to its entries'
    completion); an entry completes when it and its complement head their queues (same queue models as
    :func:`simulate`), ``comm`` after the later of the two posts.  Returns the makespan, per-stage busy
    time, the bubble fraction 1 - busy / (S * makespan), and every wait's idle gap (stage, item index,
    clock before the wait, completion time)."""
    S = len(progs)
    pc = [0] * S
    clock = [0.0] * S
    busy = [0.0] * S
    queues: Dict[Tuple[int, int], List[tuple]] = {}
    done: Dict[Tuple[int, str], float] = {}
    gaps: List[tuple] = []
    while True:
        progressed = False
        for s in range(S):
            while pc[s] < len(progs[s]):
                it = progs[s][pc[s]]
                if it[0] == "post":
                    _, name, peer, snd, rcv = it
                    key = (s, s + peer) if model == "pair" else (s, -1)
                    queues.setdefault(key, []).append((name, frozenset(snd), frozenset(rcv), s + peer, clock[s]))
                elif it[0] == "wait":
                    if not all((s, n) in done for n in it[1]):
                        break
                    t = max(done[(s, n)] for n in it[1])
                    if t > clock[s]:
                        gaps.append((s, pc[s], clock[s], t))
                    clock[s] = max(clock[s], t)
                else:
                    c = costs[s].get(it[0], 0.0)
                    clock[s] += c
                    busy[s] += c
                pc[s] += 1
                progressed = True
        for (a, _), qa in list(queues.items()):
            while qa:
                b = qa[0][3]
                qb = queues.get((b, a) if model == "pair" else (b, -1), [])
                if not qb or qb[0][3] != a:
                    break
                na, sa, ra, _, ta = qa[0]
                nb, sb, rb, _, tb = qb[0]
                if sa != rb or ra != sb:
                    raise RuntimeError(f"timeline: message order mismatch at stages {a}/{b} ({na} vs {nb})")
                qa.pop(0)
                qb.pop(0)
                t = max(ta, tb) + _comm_cost(comm, sa | ra)
                done[(a, na)] = t
                done[(b, nb)] = t
                progressed = True
        if all(pc[s] == len(progs[s]) for s in range(S)):
            span = max(clock)
            bubble = 1.0 - sum(busy) / (S * span) if span > 0 else 0.0
            return {"makespan": span, "busy": busy, "bubble": bubble, "gaps": gaps, "end": clock}
        if not progressed:
            raise RuntimeError("timeline: deadlock")


def w_cap(S: int, s: int) -> int:
    """Most W's stage s may hold pending (each keeps its microbatch's weight-gradient operands, dY and X,
    alive): S, the number of microbatches 1F1B keeps in flight on its first stage -- ZB-H1's bound, which
    keeps every stage's peak within 1F1B's peak stage (a pending W holds less than an in-flight
    microbatch's activations).  A tighter per-stage S - s costs the 8 x 8 replay 19 % (10.3 -> 12.3)."""
    return max(1, S)


def max_pending_w(prog: List[tuple]) -> int:
    """Largest number of microbatches whose B has run and whose W has not, over a stage program."""
    pend = peak = 0
    for it in prog:
        if it[0] == "B":
            pend += 1
            peak = max(peak, pend)
        elif it[0] == "W":
            pend -= 1
    return peak


def _place_w(progs, base, s, costs, comm, M):
    """Stage s's program with its W's moved out of the steady state into the idle gaps the timed replay
    shows (the other stages as in ``progs``), the ones that fit nowhere at the end -- but never more than
    :func:`w_cap` pending: a B that would exceed it runs the oldest pending W right after itself."""
    prog = base[s]
    cap = w_cap(len(progs), s)
    trial = list(progs)
    trial[s] = prog + [("W", i) for i in range(M)]
    tl = timeline(trial, costs, comm)
    gap_at = {idx: (t0, t1) for (st, idx, t0, t1) in tl["gaps"] if st == s}
    wcost = costs[s]["W"]
    ws: List[int] = []
    out: List[tuple] = []
    delay = 0.0  # how far the W's placed so far pushed this stage's clock past the replay's
    for idx, it in enumerate(prog):
        if it[0] != "post":  # over the cap: the oldest W's run now, after the B's own message posts
            while len(ws) >= cap:
                out.append(("W", ws.pop(0)))
                delay += wcost
        if it[0] == "wait" and idx in gap_at:
            t0, t1 = gap_at[idx]
            room = (t1 - t0) - delay
            while ws and wcost <= room + 1e-9:
                out.append(("W", ws.pop(0)))
                room -= wcost
            delay = max(0.0, delay - (t1 - t0))
        out.append(it)
        if it[0] == "B":
            ws.append(it[1])
    tail = [("W", i) for i in ws]
    if out and out[-1][0] == "wait":  # before the final wait on the stage's sends
        return out[:-1] + tail + [out[-1]]
    return out + tail


def zb_programs(S: int, M: int, costs=None, comm: float = 0.0, head_split: bool = False) -> List[List[tuple]]:
    """ZB-H1-style programs: 1F1B's items with every B split into B (input gradients) and W (weight
    gradients), W placed to fill idle time.  Start from 1F1B with a split backward (each W right after
    its B: 1F1B's timing); then stage by stage the W's leave the steady state for the idle gaps of the
    timed replay (:func:`_place_w`).  The placement depends on the order the stages are visited in (a
    placed W changes when its stage posts later messages): first-to-last, last-to-first and a second
    pass of each are tried and the programs with the shortest replayed makespan are kept.  Memory stays
    within 1F1B's peak: a W never moves before its own B, and at most ``w_cap(S, s)`` = S W's (their dY / X
    operands) are pending on any stage at any time -- the number of microbatches 1F1B keeps in flight on
    its first stage (``tests/test_pp_schedule_cpu.py`` checks it for S up to 8 and M up to 32)."""
    costs = stage_item_costs(S) if costs is None else costs
    base = [pp_program("1f1b", S, s, M, head_split=head_split) for s in range(S)]
    inline = [[x for it in b for x in ((it, ("W", it[1])) if it[0] == "B" else (it,))] for b in base]
    if S == 1:
        return inline
    best, best_t = inline, timeline(inline, costs, comm)["makespan"]
    # starting states: 1F1B timing (W inline) and the W-free pipeline (the other stages' W's not yet
    # placed count as free while a stage is placed)
    for start, order in ((inline, list(range(S))), (inline, list(reversed(range(S)))), (base, list(range(S))),
                         (base, list(reversed(range(S))))):
        progs = [list(p) for p in start]
        for _ in range(2):
            for s in order:
                progs[s] = _place_w(progs, base, s, costs, comm, M)
            t = timeline(progs, costs, comm)["makespan"]
            if t < best_t - 1e-9:
                best, best_t = [list(p) for p in progs], t
    return best


def estimate(kind: str, S: int, M: int, costs=None, comm: float = 0.0, head_split: bool = False) -> Dict[str, float]:
    """Predicted step (makespan) and bubble of a schedule under per-item costs (``stage_item_costs``):
    the 1F1B / GPipe B items cost B + W (their backward runs the weight gradients inline)."""
    costs = stage_item_costs(S) if costs is None else costs
    if kind == "zb":
        progs = zb_programs(S, M, costs, comm, head_split=head_split)
        c = costs
    else:
        progs = [pp_program(kind, S, s, M, head_split=head_split) for s in range(S)]
        c = [dict(x, B=x["B"] + x["W"], W=0.0) for x in costs]
    tl = timeline(progs, c, comm)
    return {"makespan": tl["makespan"], "bubble": tl["bubble"], "ideal": max(M * sum(x.values()) for x in costs)}


def simulate(kind: str, S: int, M: int, model: str = "pair", head_split: bool = False) -> Dict[str, int]:
    """Run every stage's :func:`pp_program` under RCCL p2p semantics and return counters.

    Model: each stage executes its items in order on one compute stream; a ``post`` enqueues its
    entry once every earlier compute item of the stage is done (the comm stream waits on the compute
    stream); a ``wait`` blocks the stage until its entries completed.  Queues:

    * ``model="pair"``: one ordered queue per (stage, peer) pair -- the heads of the two queues of a
      pair complete TOGETHER when both are posted and complementary (sends of one == receives of
      the other, as sets: a grouped call);
    * ``model="rank"``: ONE ordered queue per stage for all its peers -- what PyTorch's coalesced p2p
      does on RCCL (every ``batch_isend_irecv`` of a group is one kernel on the group communicator's
      single stream, so a stage's posts to s-1 and to s+1 serialise in issue order).  A head entry
      completes only when the peer's head entry is its complement.

    Raises RuntimeError on a deadlock or on a head pair that does not match (wrong message order)."""
    if model not in ("pair", "rank"):
        raise ValueError(model)
    hk = {"head_split": True} if head_split else {}
    progs = zb_programs(S, M, **hk) if kind == "zb" else [pp_program(kind, S, s, M, **hk) for s in range(S)]
    pc = [0] * S
    queues: Dict[Tuple[int, int], List[tuple]] = {}
    done = set()
    counts = {"posts": 0, "waits": 0, "compute": 0}
    while True:
        progressed = False
        for s in range(S):
            while pc[s] < len(progs[s]):
                it = progs[s][pc[s]]
                if it[0] == "post":
                    _, name, peer, snd, rcv = it
                    key = (s, s + peer) if model == "pair" else (s, -1)
                    queues.setdefault(key, []).append((name, frozenset(snd), frozenset(rcv), s + peer))
                    counts["posts"] += 1
                elif it[0] == "wait":
                    if not all((s, n) in done for n in it[1]):
                        break
                    counts["waits"] += 1
                else:
                    counts["compute"] += 1
                pc[s] += 1
                progressed = True
        for (a, b), qa in list(queues.items()):
            while qa:
                b = qa[0][3]  # the head entry's peer
                qb = queues.get((b, a) if model == "pair" else (b, -1), [])
                if not qb or qb[0][3] != a:
                    break  # rank model: the peer's stream is busy with another peer first
                na, sa, ra, _ = qa[0]
                nb, sb, rb, _ = qb[0]
                if sa != rb or ra != sb:
                    # two sends (or two receives) at the heads of a pair wait on each other forever
                    what = "deadlock (head-of-line)" if (sa and sb and not (ra or rb)) or (ra and rb and not (
                        sa or sb)) else "message order mismatch"
                    raise RuntimeError(f"{kind} S={S} M={M}: {what}: stage {a} entry {na} sends {sorted(sa)} "
                                       f"receives {sorted(ra)}, stage {b} entry {nb} sends {sorted(sb)} "
                                       f"receives {sorted(rb)}")
                qa.pop(0)
                qb.pop(0)
                done.add((a, na))
                done.add((b, nb))
                progressed = True
        if all(pc[s] == len(progs[s]) for s in range(S)):
            left = {k: v for k, v in queues.items() if v}
            if left:
                raise RuntimeError(f"{kind} S={S} M={M}: unmatched entries at the end: {left}")
            return counts
        if not progressed:
            stuck = {s: progs[s][pc[s]] for s in range(S) if pc[s] < len(progs[s])}
            raise RuntimeError(f"{kind} S={S} M={M}: deadlock, stages blocked at {stuck}")


# ------------------------------------------------------------------------------ executor
class _HostSend:
    """isend of a device tensor through a host copy (gloo backend); ``wait()`` like a Work."""

    def __init__(self, t, dst):
        self.host = t.detach().to("cpu")
        self.work = dist.isend(self.host, dst)

    def wait(self):
        self.work.wait()
        self.host = None


def _host_recv(buf, src):
    host = torch.empty(buf.shape, dtype=buf.dtype)
    dist.recv(host, src)
    buf.copy_(host)


def run_pipeline(eng) -> None:
    m = eng.mesh
    st = eng.stage
    prog = eng.program
    S, s, M = m.pp, m.pp_idx, eng.n_micro
    T, rows = eng.T, eng.mb_rows
    first, last = s == 0, s == S - 1
    step = eng.opt.step_t
    ctxs: Dict[int, Dict] = {i: {} for i in range(M)}
    grad_scale = 1.0 / (rows * T * M * m.dp)
    loss_scale = 1.0 / (rows * T * M)
    n_bwd_done = 0
    if not last:
        fill_(eng.loss, 0.0)
    staged = staged_p2p() and eng.device.type == "cuda"
    outs: Dict[int, torch.Tensor] = {}  # forward outputs (sent to the next stage)

    bf = getattr(eng, "pp_bf16", False)  # bf16 stage messages (pp_comm_dtype): the bf16 images travel
    hs = bool(getattr(eng, "pp_head_split", False))
    head_a, head_b = hs and s == S - 2, hs and s == S - 1  # the two halves of a split head

    def tensor_of(tag, sending):
        d, i = tag
        if d == "s":  # head split: packed row statistics of the half (both directions)
            return ctxs[i]["head_stats"] if sending else eng.recv_s[i]
        if d == "f" and (head_a if sending else head_b):  # the final LayerNorm output, compute dtype
            return outs[i] if sending else eng.recv_yf[i]
        if bf:
            if d == "f":
                return eng.send_x_bf[i] if sending else eng.recv_x_bf[i]
            return eng.send_dx_bf[i] if sending else eng.recv_dx_bf[i]
        if d == "f":
            return outs[i] if sending else eng.recv_x[i]
        return dx_out[i] if sending else eng.recv_dx[i]

    def issue(peer, snd, rcv):
        """One grouped p2p call; snd / rcv are tensors (resolved when the program runs, so a replayed
        hipGraph step moves the same buffers)."""
        rank = m.pp_next if peer > 0 else m.pp_prev
        if staged:  # gloo carries host tensors only: host-staged sends, blocking host receives
            works = [_HostSend(t, rank) for t in snd]
            for t in rcv:
                _host_recv(t, rank)
            return works
        ops = [dist.P2POp(dist.isend, t, rank) for t in snd]
        ops += [dist.P2POp(dist.irecv, t, rank) for t in rcv]
        return dist.batch_isend_irecv(ops)

    def run_comm(run):
        """Every p2p item between two compute items in ONE collective call (one graph cut): posts
        whose wait is in the same run are waited right away, the others are parked by name."""
        waited_here = {n for it in run if it[0] == "wait" for n in it[1]}
        steps = []
        for it in run:
            if it[0] == "post":
                _, name, peer, snd, rcv = it
                steps.append(("post", name, peer, [tensor_of(t, True) for t in snd],
                              [tensor_of(t, False) for t in rcv]))
            else:
                steps.append(it)
        local = {}
        replayed = prog.recording  # a recorded item is re-run by every replay: it must keep its tensors

        def release(name):
            """Eager steps: a send whose post was waited no longer needs its buffer -- drop the stage's
            references (forward output / input gradient), so 1F1B holds ~S microbatches, not M."""
            if replayed:
                return
            for d, i in sent_tags.get(name, ()):  # (the post may belong to an earlier run)
                (outs if d == "f" else dx_out).pop(i, None)

        def fn():
            for st_ in steps:
                if st_[0] == "post":
                    _, name, peer, snd, rcv = st_
                    works = issue(peer, snd, rcv)
                    if name in waited_here:
                        local[name] = works
                    else:
                        prog._handles[name] = works
                else:
                    for n in st_[1]:
                        if n in local:
                            for w in local.pop(n):
                                w.wait()
                        else:
                            prog._wait(n)
                        release(n)

        sig = []
        for st_ in steps:
            if st_[0] == "post":
                _, _, peer, snd, rcv = st_
                rank = m.pp_next if peer > 0 else m.pp_prev
                sig += [x for t in snd for x in psig("send", rank, t)] + [x for t in rcv for x in psig("recv", rank, t)]
        # PP point-to-point stays eager between segments (RCCL p2p inside a capture is unexercised here)
        prog.comm(fn, sig=sig, capturable=False)

    kind = eng.tcfg.pp_schedule
    zb = kind == "zb"
    items = pp_program(kind, S, s, M, costs=eng.pp_item_costs() if zb else None, head_split=hs,
                       comm=eng.pp_comm_costs() if zb else 0.0)
    wq: Dict[int, list] = {}  # zb: microbatch -> its queued weight gradients (run by its W item)
    n_w_done = 0
    sent_tags = {it[1]: it[3] for it in items if it[0] == "post"}  # post name -> tags it sends
    dx_out: Dict[int, torch.Tensor] = {}
    k = 0
    while k < len(items):
        if items[k][0] in ("post", "wait"):
            j = k
            while j < len(items) and items[j][0] in ("post", "wait"):
                j += 1
            run_comm(items[k:j])
            k = j
            continue
        kind, i = items[k]
        if kind == "W":
            st.run_wgrads(wq.pop(i), 0.0 if n_w_done == 0 else 1.0)
            n_w_done += 1
            k += 1
            continue
        ids = eng.ids[i * rows:(i + 1) * rows]
        labels = eng.labels[i * rows:(i + 1) * rows]
        row0 = eng.row0 + i * rows
        ctx = ctxs[i]
        if kind == "H":  # head split: this stage's vocab half (A reads its own LayerNorm output)
            st.head_split_logits(eng.recv_yf[i] if head_b else None, labels, ctx)
            k += 1
            continue
        if kind == "Hf":
            st.head_split_finalize(ctx, eng.recv_s[i], loss_scale, loss_out=eng.loss if last else None,
                                   accumulate=(i > 0))
            k += 1
            continue
        if kind == "F":
            if not first and bf:
                cast_bf16_to_f32(eng.recv_x_bf[i], eng.recv_x[i])
            h = st.embed_forward(ids, step, row0, ctx) if first else eng.recv_x[i]
            h = st.stage_forward(h, rows, ctx)
            if head_a:
                outs[i] = st.head_split_input(h, ctx)  # the f message to the other half
            elif last:
                st.head_forward(h, labels, loss_scale, ctx, loss_out=eng.loss, accumulate=(i > 0))
            else:
                outs[i] = h
                if bf:
                    cast_to_bf16(h, eng.send_x_bf[i])
        else:
            beta = 0.0 if n_bwd_done == 0 else 1.0
            n_bwd_done += 1
            if head_b:  # this half's input-gradient partial is the b message
                dx, _ = st.head_backward(ctx, grad_scale, beta)
                dx_c = dx
            elif last:
                dx, dx_c = st.head_backward(ctx, grad_scale, beta)
            else:
                dx = eng.recv_dx[i]
                dx_c = eng.recv_dx_c[i]
                if bf:  # the received bf16 image is the compute-dtype copy; the fp32 one is cast from it
                    cast_bf16_to_f32(eng.recv_dx_bf[i], dx)
                    if dx_c is not dx:
                        dx_c = eng.recv_dx_bf[i]
                elif dx_c is not dx and not head_a:
                    cast_to_bf16(dx, dx_c)
                if head_a:  # the other half's partial joins this half's before the final LayerNorm backward
                    dx, dx_c = st.head_backward(ctx, grad_scale, beta, extra_dyf=dx)
            dx, dx_c = st.stage_backward(ctx, dx, dx_c, beta, keep_wgrads=zb)
            if zb:
                wq[i] = st.take_wgrads()
            if first:
                st.embed_backward(ctx, dx, step, beta)
            else:
                dx_out[i] = dx
                if bf:
                    cast_to_bf16(dx, eng.send_dx_bf[i])
        k += 1
