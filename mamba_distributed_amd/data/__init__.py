from .loader import DataLoaderLite, SyntheticTokens, load_tokens, write_synthetic_shards

__all__ = ["DataLoaderLite", "SyntheticTokens", "load_tokens", "write_synthetic_shards"]
