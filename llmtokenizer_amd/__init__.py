"""llmtokenizer_amd -- MI355X-native (gfx950) byte-pair-encoding trainer,
encoder and decoder behind the C API of neofytr/LLMTokenizer (include/bpe.h).

The product is the C-ABI library libbpe_amd.so (HIP kernels + C host code);
this package is its Python binding plus the synthetic-corpus generator.
"""
from .api import (BpeError, Engine, compress, decompress, device_count, dump_pairs, encode,  # noqa: F401
                  last_stats, read_pairs, train_bytes)
from .synth import synth_bytes  # noqa: F401
