"""mimi_hip — MI355X-native Mimi encode engine (drop-in for the potsawee/tokenize-audio encode path).

    from mimi_hip import MimiEncoder                 # replaces the scripts' `class MimiEncoder`
    from mimi_hip import MimiHipModel                # replaces transformers.MimiModel for .encode
    from mimi_hip import codes_to_chars              # replaces utils.codes_to_chars

torch is imported lazily by the model modules; ``mimi_hip.config`` / ``mimi_hip.synthetic`` / ``mimi_hip.codes``
need only numpy.
"""
from .config import MimiConfig, encoded_length  # noqa: F401

__all__ = ["MimiConfig", "encoded_length", "MimiHipModel", "MimiEncoderOutput", "MimiEncoder",
           "MimiFeatureExtractor", "codes_to_chars", "chars_to_codes", "audio_to_str"]


def __getattr__(name):
    if name in ("MimiHipModel", "MimiEncoderOutput"):
        from . import model
        return getattr(model, name)
    if name == "MimiEncoder":
        from .encoder import MimiEncoder
        return MimiEncoder
    if name == "MimiFeatureExtractor":
        from .feature_extraction import MimiFeatureExtractor
        return MimiFeatureExtractor
    if name in ("codes_to_chars", "chars_to_codes", "audio_to_str"):
        from . import codes
        return getattr(codes, name)
    raise AttributeError(name)
