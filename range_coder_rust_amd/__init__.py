"""range_coder_rust_amd — MI355X-native batched range coder (drop-in for the encode/decode path
of diegodox/range_coder_rust).  See DESIGN.md and include/range_coder.h."""
from .api import (  # noqa: F401
    ADAPTIVE_DEFAULTS, AdaptiveModel, BadSymbolError, CapacityError, ChunkTooLongError, Context, CorruptStreamError, Decoder, Encoder, FreqTable,
    PModel, RangeCoderError, StaticModel, TruncatedStreamError, ZeroFrequencyError,
    decode_batch, decode_chunks, default_context, encode_batch, encode_chunks, flag_names,
    slot_capacity, encode_host, decode_host, BadModelError, ByteCount, FinishedError, RangeCoder,
    LowerBoundOverflow, UpperBoundOverflow,
    stream_states, stream_encode_batch, stream_decode_batch, encode_host_multi, decode_host_multi,
)
from . import synth  # noqa: F401
from .model_build import build_model, histogram, ideal_bits, quantize_counts  # noqa: F401
from . import container  # noqa: F401
from .container import ContainerError, compress, decompress  # noqa: F401

__version__ = "0.1.0"
