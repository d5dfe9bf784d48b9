"""Model families: Mamba-1 (S6) and Mamba-2 (SSD) LMs, plus hybrid attention / MLP layers."""
from .layers import MHA, GatedMLP
from .mamba1 import Mamba
from .mamba2 import Mamba2
from .mixer_seq import (Block, CausalLMOutput, InferenceParams, MambaLMHeadModel, MixerModel,
                        create_block)

__all__ = ["MHA", "GatedMLP", "Mamba", "Mamba2", "Block", "CausalLMOutput", "InferenceParams",
           "MambaLMHeadModel", "MixerModel", "create_block"]
