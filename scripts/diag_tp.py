"""Diagnose GPU tensor-parallel numerics: per-parameter gradient error of a TP=2 run (2 ranks on
one GPU over gloo) against the single-GPU model, after one forward+backward."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset  # noqa
from distributed_training_compare_jax_amd.data.synthetic import get_batch_iterator  # noqa
from distributed_training_compare_jax_amd.parallel.dist import DistInfo, spawn  # noqa

MC = model_config_from_preset("tiny", vocab_size=1000, n_layers=2)


def fwd_bwd(eng):
    b = next(get_batch_iterator(4, MC.max_seq_len + 1, vocab=999))
    eng.set_batch(b)
    st, T = eng.stage, MC.max_seq_len
    ctx = {}
    h = st.embed_forward(eng.ids, eng.opt.step_t, 0, ctx)
    h = st.stage_forward(h, 4, ctx)
    loss = st.head_forward(h, eng.labels, 1 / (4 * T), ctx)
    dx, dxc = st.head_backward(ctx, 1 / (4 * T), 0.0)
    dx, dxc = st.stage_backward(ctx, dx, dxc, 0.0)
    st.embed_backward(ctx, dx, eng.opt.step_t, 0.0)
    torch.cuda.synchronize()
    return loss.item(), {n: eng.flat.g(n).cpu().clone() for n in eng.flat.slots}


def worker(out):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    from distributed_training_compare_jax_amd.parallel.dist import init_distributed
    from distributed_training_compare_jax_amd.train.engine import Engine
    d = init_distributed("cuda")
    tc = TrainConfig(seed=0, parallel="tp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=False)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), d)
    loss, g = fwd_bwd(eng)
    torch.save({"loss": loss, "g": g}, os.path.join(out, f"r{d.rank}.pt"))


def main():
    from distributed_training_compare_jax_amd.models.params import all_param_specs, unshard
    from distributed_training_compare_jax_amd.train.engine import Engine
    with tempfile.TemporaryDirectory() as td:
        spawn(worker, 2, args=(td,))
        rs = [torch.load(os.path.join(td, f"r{i}.pt")) for i in range(2)]
    tc = TrainConfig(seed=0, parallel="dp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=False)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0),
                 DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl"))
    loss, g = fwd_bwd(eng)
    print("loss single", loss, "tp", rs[0]["loss"], rs[1]["loss"])
    specs = {s.name: s for s in all_param_specs(MC)}
    for n in g:
        full = unshard(specs[n], [rs[0]["g"][n], rs[1]["g"][n]])
        err = ((full - g[n]).norm() / (g[n].norm() + 1e-12)).item()
        print(f"{n:14s} rel err {err:.3e}", "  <-- BAD" if err > 5e-2 else "")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def worker_step(out):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    from distributed_training_compare_jax_amd.parallel.dist import init_distributed
    from distributed_training_compare_jax_amd.train.engine import Engine
    d = init_distributed("cuda")
    tc = TrainConfig(seed=0, parallel="tp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=False)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), d)
    b = next(get_batch_iterator(4, MC.max_seq_len + 1, vocab=999))
    eng.set_batch(b)
    eng.run_step()
    torch.cuda.synchronize()
    torch.save({"loss": eng.loss_value(), "ss": eng.opt.sumsq.item(), "step": eng.opt.step_t.item(),
                "p": {n: eng.flat.p(n).cpu().clone() for n in eng.flat.slots},
                "segs": eng.opt.segments.cpu()}, os.path.join(out, f"s{d.rank}.pt"))


def main_step():
    from distributed_training_compare_jax_amd.models.params import all_param_specs, unshard
    from distributed_training_compare_jax_amd.train.engine import Engine
    with tempfile.TemporaryDirectory() as td:
        spawn(worker_step, 2, args=(td,))
        rs = [torch.load(os.path.join(td, f"s{i}.pt")) for i in range(2)]
    tc = TrainConfig(seed=0, parallel="dp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=False)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0),
                 DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl"))
    b = next(get_batch_iterator(4, MC.max_seq_len + 1, vocab=999))
    eng.set_batch(b)
    eng.run_step()
    torch.cuda.synchronize()
    print("sumsq single", eng.opt.sumsq.item(), "tp", rs[0]["ss"], rs[1]["ss"], "steps", rs[0]["step"])
    print("segments rank0", rs[0]["segs"][:6].tolist(), len(rs[0]["segs"]))
    specs = {s.name: s for s in all_param_specs(MC)}
    for n in eng.flat.slots:
        full = unshard(specs[n], [rs[0]["p"][n], rs[1]["p"][n]])
        ref = eng.flat.p(n).cpu()
        err = ((full - ref).norm() / (ref.norm() + 1e-12)).item()
        print(f"{n:14s} param rel err {err:.3e}", "  <-- BAD" if err > 1e-3 else "")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "step":
    main_step()


def worker_graph(out, use_graph):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    from distributed_training_compare_jax_amd.parallel.dist import init_distributed
    from distributed_training_compare_jax_amd.train.engine import Engine
    d = init_distributed("cuda")
    tc = TrainConfig(seed=0, parallel="tp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=use_graph)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), d)
    it = get_batch_iterator(4, MC.max_seq_len + 1, vocab=999)
    rec = []
    for i in range(4):
        eng.set_batch(next(it))
        eng.run_step()
        torch.cuda.synchronize()
        rec.append((eng.loss_value(), eng.opt.sumsq.item(), eng.flat.p("h.0.fc1.w").float().norm().item(),
                    eng.flat.mirror[:1000].float().norm().item()))
    if d.rank == 0:
        print("graph" if use_graph else "eager", [tuple(round(v, 5) for v in r) for r in rec], flush=True)
        print("items", [(k, n) for k, _, n in eng.program.items][:40], flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "graph":
    with tempfile.TemporaryDirectory() as td:
        spawn(worker_graph, 2, args=(td, False))
        spawn(worker_graph, 2, args=(td, True))


def worker_graph2(out):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    from distributed_training_compare_jax_amd.parallel.dist import init_distributed
    from distributed_training_compare_jax_amd.train.engine import Engine
    d = init_distributed("cuda")
    tc = TrainConfig(seed=0, parallel="tp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=True)
    eng = Engine(MC, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), d)
    it = get_batch_iterator(4, MC.max_seq_len + 1, vocab=999)
    for i in range(4):
        eng.set_batch(next(it))
        eng.run_step()
        torch.cuda.synchronize()
        g = eng.flat.grads
        bad = [n for n in eng.flat.slots if not torch.isfinite(eng.flat.g(n)).all()]
        segs = eng.opt.segments.cpu()
        w = sum(float(wt) * float((g[int(o):int(o) + int(n_)].double() ** 2).sum()) for o, n_, wt in segs.tolist())
        if d.rank == 0:
            print(i, "sumsq", eng.opt.sumsq.item(), "torch local weighted", w, "nonfinite grads:", bad,
                  "gmax", g.abs().max().item(), [(n, eng.flat.g(n).abs().max().item()) for n in ('wte', 'wpe')], flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "graph2":
    with tempfile.TemporaryDirectory() as td:
        spawn(worker_graph2, 2, args=(td,))
