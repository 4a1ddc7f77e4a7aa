"""MI355X-native HiFi-GAN Generator inference path (drop-in for
terrense/TTS-sambert_hifiGAN ``models/hifigan.py`` Generator.forward).

The directory name contains a hyphen, so import it with :func:`load_package`
from the repo root (``__graft_entry__``, ``bench.py`` and ``tests/conftest.py``
do this), which registers it as ``tts_sambert_hifigan_amd``.
"""
from .hifigan import HiFiGAN, HiFiGANGenerator, MRF, ResBlock, get_padding  # noqa: F401
from ._lib import (HipExtensionMissing, HfgError, Handle, load_library, make_config,  # noqa: F401
                   LIB_PATH, check_provenance, schedule_override, schedule_clear,
                   schedule_overrides)

__all__ = ["HiFiGAN", "HiFiGANGenerator", "MRF", "ResBlock", "get_padding", "Handle",
           "HipExtensionMissing", "HfgError", "load_library", "make_config", "LIB_PATH", "check_provenance",
           "schedule_override", "schedule_clear", "schedule_overrides"]
