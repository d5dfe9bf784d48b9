"""mamba_distributed_amd — an MI355X-native (gfx950 / CDNA4) Mamba-1 / Mamba-2 training framework.

Layers:
  config.MambaConfig / lm.LMHeadModel     model API (reference model.py)
  models/                                  Mamba1, Mamba2, Block, MixerModel, LM head, MHA/MLP
  ops/                                     autograd ops -> HIP kernels (csrc/kernels/*.hip) | torch refs
  parallel/                                torch.distributed over RCCL/xGMI: DDP, context parallel
  data/                                    token shards, synthetic data, native prefetcher
  utils/                                   checkpoints, logging, LR schedule, profiling, tokenizer
"""
from .config import MambaConfig, preset
from .lm import LMHeadModel
# mamba-ssm's top-level names (``from mamba_ssm import Mamba, Mamba2, MambaLMHeadModel``)
from .models.mamba1 import Mamba
from .models.mamba2 import Mamba2
from .models.mixer_seq import MambaLMHeadModel

__version__ = "0.1.0"
__all__ = ["MambaConfig", "preset", "LMHeadModel", "Mamba", "Mamba2", "MambaLMHeadModel"]
