"""Importable name of the package that lives in ``tts-sambert_hifigan_amd/``.

The source directory's name carries a hyphen (the project layout), which Python
cannot import directly.  This shim makes ``import tts_sambert_hifigan_amd`` (with
the repo root on ``sys.path``) resolve every submodule from that directory: it
points the package ``__path__`` there and runs its ``__init__``.  Nothing else
lives here.
"""
import os as _os

_REAL = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "tts-sambert_hifigan_amd")
__path__ = [_REAL]
__file__ = _os.path.join(_REAL, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
