"""CLI entry point — same interface as the reference ``main.py:10-57``.

    python main.py --train_config_path configs/train_config_{dp,tp,pp}.yaml

Loads ``configs/model_config.yaml`` and ``configs/optim_config.yaml`` (paths relative to the
CWD, as in the reference), injects ``vocab_size`` (50258 = GPT-2 + <pad>) and
``parallel``, prints ``Running `<strategy>` on N devices.`` and trains.

Process model: one rank per GPU.  Under ``torchrun`` the ranks already exist; started as
a plain script it spawns one process per visible GPU itself (the reference uses every
visible device, ``main.py:34``).  ``--nproc`` overrides the count (e.g. gloo ranks on CPU).
"""

from __future__ import annotations

import os

import click


def _run(train_config_path: str, model_config_path: str, optim_config_path: str, overrides: dict):
    from distributed_training_compare_jax_amd.config.schema import build_configs, replace
    from distributed_training_compare_jax_amd.data.synthetic import get_tokenizer
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.train.loop import train

    train_config, model_config, opt_config = build_configs(train_config_path, model_config_path, optim_config_path,
                                                           vocab_size=len(get_tokenizer()))
    if overrides:
        train_config = replace(train_config, **overrides)
    if train_config.parallel not in ("dp", "tp", "pp"):
        raise ValueError(f"Unsupported strategy `{train_config.parallel}`")
    dinfo = init_distributed(train_config.device)
    if dinfo.rank == 0:
        print(f"Running `{train_config.parallel}` on {dinfo.world} devices.", flush=True)
    try:
        train(train_config, model_config, opt_config, dinfo)
    finally:
        destroy()


def _parse_sets(items) -> dict:
    """KEY=VALUE strings -> TrainConfig overrides, each value parsed as its field's type."""
    import dataclasses

    from distributed_training_compare_jax_amd.config.schema import TrainConfig

    types = {f.name: str(f.type) for f in dataclasses.fields(TrainConfig)}
    out = {}
    for it in items:
        k, v = it.split("=", 1)
        if k not in types:
            raise click.BadParameter(f"unknown TrainConfig field {k!r}", param_hint="--set")
        t = types[k]
        if v.lower() in ("none", "null") and "Optional" in t:
            out[k] = None
        elif "bool" in t:
            out[k] = v.lower() in ("1", "true", "yes")
        elif "int" in t:
            out[k] = int(v)
        elif "float" in t:
            out[k] = float(v)
        else:
            out[k] = v
    return out


def _spawn_target(args):
    _run(*args)


@click.command()
@click.option("--train_config_path", default="configs/train_config_dp.yaml")
@click.option("--model_config_path", default="configs/model_config.yaml", show_default=True)
@click.option("--optim_config_path", default="configs/optim_config.yaml", show_default=True)
@click.option("--nproc", type=int, default=None, help="ranks to spawn (default: all visible GPUs, else 1)")
@click.option("--steps", type=int, default=None, help="override train_config.steps")
@click.option("--device", type=click.Choice(["auto", "cuda", "cpu"]), default=None)
@click.option("--log_every", type=int, default=None, help="override train_config.log_every")
@click.option("--warmup_steps", type=int, default=None, help="override the 5 untimed warmup steps")
@click.option("--output_dir", default=None, help="override train_config.output_dir")
@click.option("--profile", is_flag=True, default=False,
              help="roctx ranges + device step times + Chrome trace in <output_dir>/trace/")
@click.option("--dtype", type=click.Choice(["bf16", "fp32"]), default=None,
              help="compute precision (default bf16; fp32 = the reference's precision on the exact-fp32 kernels)")
@click.option("--set", "sets", multiple=True, metavar="KEY=VALUE",
              help="any other TrainConfig field, e.g. --set tp_comm=p2p --set pp_schedule=1f1b")
def main(train_config_path: str, model_config_path: str, optim_config_path: str, nproc, steps, device, log_every,
         warmup_steps, output_dir, profile, dtype, sets):
    overrides = _parse_sets(sets)
    if dtype is not None:
        overrides["dtype"] = dtype
    if output_dir is not None:
        overrides["output_dir"] = output_dir
    if profile:
        overrides["profile"] = True
    if steps is not None:
        overrides["steps"] = steps
    if log_every is not None:
        overrides["log_every"] = log_every
    if warmup_steps is not None:
        overrides["warmup_steps"] = warmup_steps
    if device is not None:
        overrides["device"] = device
    args = (train_config_path, model_config_path, optim_config_path, overrides)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        _run(*args)
        return
    import torch

    if nproc is None:
        nproc = torch.cuda.device_count() if (device != "cpu" and torch.cuda.device_count() > 0) else 1
    if nproc <= 1:
        _run(*args)
        return
    from distributed_training_compare_jax_amd.parallel.dist import spawn

    spawn(_spawn_target, nproc, args=(args,))


if __name__ == "__main__":
    main()
