"""MI355X-native distributed GPT training comparison (DP vs TP vs PP).

A from-scratch re-design of KT19/distributed-training-compare-jax for AMD Instinct
MI355X (gfx950): PyTorch-ROCm process-per-GPU runtime, hand-written HIP/CDNA4 kernels
(``csrc/``), RCCL collectives over xGMI, hipGraph-captured training steps.
"""

__version__ = "0.1.0"
