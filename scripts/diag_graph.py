import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
from distributed_training_compare_jax_amd.data.synthetic import get_batch_iterator
from distributed_training_compare_jax_amd.parallel.dist import DistInfo
from distributed_training_compare_jax_amd.train.engine import Engine
dev = torch.device("cuda", 0)
preset = sys.argv[1] if len(sys.argv) > 1 else "tiny"
mc = model_config_from_preset(preset, vocab_size=1000 if preset == "tiny" else 50258)
tc = TrainConfig(seed=0, parallel="dp", batch=4, steps=1, log_every=1, output_dir="/tmp/x", use_graph=True)
eng = Engine(mc, tc, OptimConfig(lr=1e-3, weight_decay=0.1, grad_clip=1.0), DistInfo(0, 1, 0, dev, "nccl"))
it = get_batch_iterator(4, mc.max_seq_len + 1, vocab=min(50256, mc.vocab_size - 1))
for i in range(4):
    eng.set_batch(next(it)); eng.run_step(); print(i, eng.loss_value(), flush=True)
