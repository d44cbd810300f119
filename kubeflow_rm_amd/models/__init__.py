"""Model families that run inside notebook pods on the framework's kernels.

* ``gpt`` — GPT-style decoder LM (MFMA GEMM with fused epilogues, LayerNorm kernel, SDPA),
  tensor-parallel aware; configs ``gpt-tiny`` / ``gpt-small`` / ``gpt-1b``.
"""
from .gpt import CONFIGS, GPT, GPTConfig, build, num_params  # noqa: F401
