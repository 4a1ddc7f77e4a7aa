"""Acoustic-model → vocoder glue and streaming vocoding.

The reference only specifies the glue (``.kiro/specs/tts-sam-bert-hifigan/design.md:905-906``:
``mel_pred.transpose(1, 2)`` then ``HiFiGAN(mel)``) and lists streaming as an
unchecked task (``requirements.md:211-220``, ``tasks.md:362``).  Both are built
here on the same HIP kernels:

* :func:`vocode_acoustic` takes ``SAMBERTAcousticModel.inference`` output
  ``[B, Tfrm, 80]`` (models/acoustic_model.py:267-297) plus per-utterance frame
  counts; the transpose is fused into conv_pre's staging and every layer
  zero-pads at the utterance's own length, so each returned wav equals the
  Generator run on that utterance alone.
* :class:`StreamingVocoder` emits audio chunk by chunk with a receptive-field
  context on both sides; the concatenated stream equals the one-shot run.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch


def vocode_acoustic(gen, mel_pred: torch.Tensor, lengths: Optional[Sequence[int]] = None
                    ) -> List[torch.Tensor]:
    """mel_pred [B, Tfrm, n_mels] (acoustic-model layout) → list of B wavs [L_b]
    with L_b = gen.output_length(lengths[b])."""
    B, T, _ = mel_pred.shape
    lens = [T] * B if lengths is None else [int(x) for x in lengths]
    wav = gen(mel_pred, lengths=lens, mel_layout="btc")
    return [wav[b, 0, :gen.output_length(lens[b])] for b in range(B)]


def vocode_list(gen, mels: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Variable-length utterances [n_mels, T_b] → list of wavs, one padded batch."""
    lens = [int(m.shape[-1]) for m in mels]
    T = max(lens)
    batch = torch.zeros(len(mels), mels[0].shape[0], T, device=mels[0].device,
                        dtype=torch.float32)
    for b, m in enumerate(mels):
        batch[b, :, :lens[b]] = m
    wav = gen(batch, lengths=lens)
    return [wav[b, 0, :gen.output_length(lens[b])] for b in range(len(mels))]


class StreamingVocoder:
    """Chunked vocoding of a growing mel stream for ONE utterance.

    ``push(frames [n_mels, t])`` returns the audio that is final so far;
    ``flush()`` returns the rest.  A chunk of ``chunk_frames`` is emitted once
    ``context`` future frames exist; it is computed from the frames
    ``[start - context, end + context)`` and cropped, so the output is identical
    to ``gen(full_mel)`` (context defaults to gen.receptive_field_frames()).
    Needs an exact-upsampling config (output length = frames × hop).
    """

    def __init__(self, gen, chunk_frames: int = 64, context: Optional[int] = None):
        self.gen = gen
        self.hop = gen.output_length(2) - gen.output_length(1)
        if gen.output_length(7) != 7 * self.hop:
            raise ValueError("streaming needs exact upsampling (out_len = T * hop)")
        self.chunk = int(chunk_frames)
        self.ctx = int(context) if context is not None else gen.receptive_field_frames()
        self.buf: Optional[torch.Tensor] = None  # all frames received [n_mels, T]
        self.emitted = 0                         # frames whose audio was returned

    def _run(self, a: int, b: int, end: int) -> torch.Tensor:
        lo, hi = max(0, a - self.ctx), min(end, b + self.ctx)
        with torch.no_grad():
            wav = self.gen(self.buf[None, :, lo:hi].contiguous())
        return wav[0, 0, (a - lo) * self.hop:(b - lo) * self.hop]

    def push(self, frames: torch.Tensor) -> torch.Tensor:
        if frames.dim() == 3:
            frames = frames[0]
        self.buf = frames if self.buf is None else torch.cat([self.buf, frames], dim=1)
        T = self.buf.shape[1]
        out = []
        while T - self.emitted >= self.chunk + self.ctx:
            a, b = self.emitted, self.emitted + self.chunk
            out.append(self._run(a, b, T))
            self.emitted = b
        return torch.cat(out) if out else self.buf.new_zeros(0)

    def flush(self) -> torch.Tensor:
        if self.buf is None:
            return torch.zeros(0)
        T = self.buf.shape[1]
        out = []
        while self.emitted < T:
            a, b = self.emitted, min(T, self.emitted + self.chunk)
            out.append(self._run(a, b, T))
            self.emitted = b
        return torch.cat(out) if out else self.buf.new_zeros(0)
