from .llama import Llama, LlamaConfig, PRESETS as LLAMA_PRESETS, build_llama

__all__ = ["Llama", "LlamaConfig", "LLAMA_PRESETS", "build_llama"]
