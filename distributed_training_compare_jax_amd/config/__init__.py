from .schema import ModelConfig, OptimConfig, TrainConfig, build_configs, model_config_from_preset  # noqa: F401
