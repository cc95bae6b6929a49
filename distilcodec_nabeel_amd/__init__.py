"""MI355X-native DistilCodec encode -> quantize -> decode path (gfx950 HIP kernels, C ABI).

Drop-in for `distilcodec.DistilCodec` (reference: nabeelscicom/DistilCodec_nabeel).  Importing the
package needs no GPU; constructing the device engine does, and fails loudly without libdcx.so.
"""
from .codec import (  # noqa: F401
    AttrDict,
    DistilCodec,
    GRVQResult,
    decode_audio,
    demo_for_generate_audio_codes,
    load_and_resample_audio,
)
from .config import default_config, load_config  # noqa: F401

__all__ = ["DistilCodec", "GRVQResult", "decode_audio", "demo_for_generate_audio_codes", "load_and_resample_audio",
           "default_config", "load_config"]
