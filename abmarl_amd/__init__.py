"""abmarl_amd — MI355X-native batched GridWorld step engine with Abmarl's API.

Product path: Python host (this package) -> C-ABI (include/gw_engine.h) ->
HIP kernels for gfx950 (abmarl_amd/csrc/gw_engine.hip).  There is no CPU
fallback: the engine raises when its library or a GPU is missing.
"""
__version__ = '0.1.0'
