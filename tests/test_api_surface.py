"""The names a mamba-ssm user imports exist here, with upstream's call shapes."""
import inspect


def test_mamba_ssm_names_importable():
    from mamba_distributed_amd import Mamba, Mamba2, MambaConfig, MambaLMHeadModel  # noqa: F401
    from mamba_distributed_amd.models.layers import MHA, GatedMLP  # noqa: F401
    from mamba_distributed_amd.models.mixer_seq import Block, InferenceParams, MixerModel, create_block  # noqa: F401
    from mamba_distributed_amd.ops import (RMSNorm, RMSNormGated, causal_conv1d_fn,  # noqa: F401
                                           causal_conv1d_update, layer_norm_fn, mamba_chunk_scan_combined,
                                           mamba_inner_fn, mamba_split_conv1d_scan_combined, rms_norm_fn,
                                           selective_scan_fn, selective_state_update)
    from mamba_distributed_amd.utils.generation import GenerationMixin, decode, sample  # noqa: F401
    assert issubclass(MambaLMHeadModel, GenerationMixin)


def test_upstream_signatures():
    from mamba_distributed_amd import Mamba2, MambaLMHeadModel
    from mamba_distributed_amd.ops import mamba_chunk_scan_combined, mamba_split_conv1d_scan_combined
    gen = inspect.signature(MambaLMHeadModel.generate).parameters
    for k in ("input_ids", "max_length", "top_k", "top_p", "min_p", "temperature", "return_dict_in_generate",
              "output_scores"):
        assert k in gen, k
    m2 = inspect.signature(Mamba2.__init__).parameters
    for k in ("d_state", "d_conv", "expand", "headdim", "d_ssm", "ngroups", "A_init_range", "D_has_hdim",
              "rmsnorm", "norm_before_gate", "dt_limit", "chunk_size", "layer_idx"):
        assert k in m2, k
    cs = inspect.signature(mamba_chunk_scan_combined).parameters
    for k in ("x", "dt", "A", "B", "C", "chunk_size", "D", "z", "dt_bias", "initial_states", "seq_idx",
              "dt_softplus", "dt_limit", "return_final_states"):
        assert k in cs, k
    sc = inspect.signature(mamba_split_conv1d_scan_combined).parameters
    for k in ("zxbcdt", "conv1d_weight", "conv1d_bias", "dt_bias", "A", "D", "chunk_size", "initial_states",
              "seq_idx", "dt_limit", "return_final_states", "activation", "rmsnorm_weight", "rmsnorm_eps",
              "outproj_weight", "outproj_bias", "headdim", "ngroups", "norm_before_gate"):
        assert k in sc, k
