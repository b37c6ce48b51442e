"""mcaat_amd — MI355X-native mcaat hot path (node_counter -> sdbg_build -> cycle_finder).

Python binding over the C ABI in include/mcaat_gpu.h (libmcaat_gpu.so, built in-tree by
`make -C mcaat_amd`). There is no CPU fallback: if the HIP library is missing or no GPU
is present, the calls raise.
"""
from .lib import (  # noqa: F401
    LIB_PATH,
    CfParams,
    Comm,
    Context,
    Counts,
    CycleResult,
    Graph,
    McaatError,
    Reads,
    SynthSpec,
    count_edges,
    edges_reduce,
    device_count,
    load_library,
    preload,
    synth_arrays,
    synth_genome_host,
    synth_host,
)
