"""Fused AdamW + transposed mirror (csrc/elementwise.hip adamw_seg_kernel / adamw_tr_kernel, DTC_ADAMW_TR):
the update over the flat buffers with the tiled weights' W^T written by the update itself must equal the
two-pass path (element-wise AdamW over everything, then the batched transpose of the fresh mirror) BITWISE --
p, m, v, the bf16 mirror and every W^T -- including edge tiles and mirror-less tails."""

import pytest
import torch

from distributed_training_compare_jax_amd.ops import optim as O

pytestmark = pytest.mark.gpu


def test_adamw_tr_matches_two_pass(cuda):
    g0 = torch.Generator().manual_seed(3)
    # (rows, cols) of the weights with a transposed mirror, laid out with gaps (biases / LN params / other
    # weights between them) as in the flat buffer; the last 4096 elements carry no mirror at all
    mats = [(768, 3072), (2304, 768), (200, 72), (96, 128)]
    gaps = [1024, 772, 4, 0, 2048]
    offs, cur = [], 0
    for (r, c), gap in zip(mats, gaps):
        cur += gap
        offs.append(cur)
        cur += r * c
    n_mirror = cur + gaps[-1]
    n = n_mirror + 4096
    p0 = torch.randn(n, generator=g0) * 0.1
    gr = torch.randn(n, generator=g0) * 0.01
    m0 = torch.randn(n, generator=g0) * 1e-3
    v0 = torch.rand(n, generator=g0) * 1e-5
    step = torch.tensor([7], dtype=torch.int64, device=cuda)
    sumsq = torch.tensor([float((gr.double() ** 2).sum()) * 4.0], dtype=torch.float32, device=cuda)  # clip active
    hp = dict(lr=3e-4, b1=0.9, b2=0.95, eps=1e-8, wd=0.1, max_norm=1.0)

    def fresh():
        return [t.clone().to(cuda) for t in (p0, gr, m0, v0)] + [torch.zeros(n_mirror, dtype=torch.bfloat16, device=cuda)]

    # two-pass reference
    p, g, m, v, mir = fresh()
    O.adamw_flat(p, g, m, v, mir, n_mirror, step, sumsq, hp["lr"], hp["b1"], hp["b2"], hp["eps"], hp["wd"],
                 hp["max_norm"])
    wts_a = [torch.zeros(c, r, dtype=torch.bfloat16, device=cuda) for r, c in mats]
    O.transpose_batch([(mir[o:o + r * c].view(r, c), t) for (r, c), o, t in zip(mats, offs, wts_a)])
    # fused
    p2, g2, m2, v2, mir2 = fresh()
    wts_b = [torch.full((c, r), 7.0, dtype=torch.bfloat16, device=cuda) for r, c in mats]
    plan = O.adamw_tr_plan(0, n, [(o, r, c, t) for (r, c), o, t in zip(mats, offs, wts_b)])
    assert plan is not None and len(plan) == 1
    O.adamw_tr(p2, g2, m2, v2, mir2, n_mirror, plan, step, sumsq, hp["lr"], hp["b1"], hp["b2"], hp["eps"], hp["wd"],
               hp["max_norm"])
    torch.cuda.synchronize()
    for a, b, name in ((p, p2, "p"), (m, m2, "m"), (v, v2, "v"), (mir, mir2, "mirror")):
        assert torch.equal(a, b), name
    for (r, c), a, b in zip(mats, wts_a, wts_b):
        assert torch.equal(a, b), (r, c)
    # and the update itself is AdamW (spot check against fp64 on the host)
    t, gc = 7.0, gr.double() * (1.0 / float(sumsq.item()) ** 0.5)
    mm = 0.9 * m0.double() + 0.1 * gc
    vv = 0.95 * v0.double() + 0.05 * gc * gc
    ref = p0.double() - 3e-4 * ((mm / (1 - 0.9 ** t)) / ((vv / (1 - 0.95 ** t)).sqrt() + 1e-8) + 0.1 * p0.double())
    assert torch.allclose(p2.cpu().double(), ref, rtol=1e-5, atol=1e-7)


def test_adamw_tr_plan_chunks_and_fallback():
    """Many weights split into several launches within the kernels' list capacities; a shape the tiled kernel
    cannot take returns None (the caller keeps the two-pass path)."""
    wt = torch.zeros(8, 8)
    mats = [(k * 200, 8, 8, wt) for k in range(150)]  # 150 tiles; 149 gaps between them + the tail
    chunks = O.adamw_tr_plan(0, 150 * 200 + 64, mats)
    assert len(chunks) == 3 and sum(tb.ntasks for _, tb in chunks) == 150
    assert sum(sb.nseg for sb, _ in chunks) == 150
    assert O.adamw_tr_plan(0, 1000, [(0, 6, 8, torch.zeros(8, 6))]) is None  # rows % 8
