"""LucyRNNConfig — the reference's configuration dataclass (lucyrnn_conf.py:3-16), verbatim API."""
from dataclasses import dataclass


@dataclass
class LucyRNNConfig:
    input_dim: int
    hidden_dim: int
    num_layers: int
    vocab_size: int
    return_last_states: bool = True
    kernel_impl: str = "native"  # 'native' or 'triton' (both run the HIP kernels here)
    is_training: bool = True      # native LucyRNN: train (scan) vs infer (step) semantics
    fused_ops: bool = False       # fused gate projections
    layer_norm: bool = True       # per-cell LayerNorms (native LucyRNN)
    stack_order: int = 1          # input frames stacked per step
    decay_mode: str = "learned"   # 'learned' or 'prefix_sum'
    lambda_decay: float = 0.001   # only for 'prefix_sum'
