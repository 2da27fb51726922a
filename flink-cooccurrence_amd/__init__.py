"""MI355X-native co-occurrence core (the non-sampled hot path of uce/flink-cooccurrence).

Import name: ``flink_cooccurrence_amd`` (the directory name has a hyphen; __graft_entry__.load_package
registers it).  Everything compute-related goes through ``csrc/libcooc_hip.so`` (include/cooc.h).
"""
from ._lib import (CoocError, HipLibraryMissing, IllegalArgumentException, IllegalStateException, header_symbols,
                   load as load_library)
from .core import (BatchResult, CooccurrenceCore, NonSampledUserInteractionCounterOneInputStreamOperator,
                   WindowResult, decode_item_cooccurrences, encode_item_cooccurrences, parse_interactions,
                   run_text_source, window_size_ms)

__all__ = [
    "BatchResult", "CoocError", "CooccurrenceCore", "HipLibraryMissing", "IllegalArgumentException",
    "IllegalStateException", "NonSampledUserInteractionCounterOneInputStreamOperator", "WindowResult",
    "decode_item_cooccurrences", "encode_item_cooccurrences", "header_symbols", "load_library",
    "parse_interactions", "run_text_source", "window_size_ms",
]
