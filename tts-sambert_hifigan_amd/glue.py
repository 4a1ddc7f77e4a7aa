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

from typing import Dict, List, Optional, Sequence

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
    """Chunked vocoding of growing mel streams with bounded state (SURVEY.md §8(f) 3;
    the reference's Requirement 18, ``.kiro/specs/tts-sam-bert-hifigan/requirements.md:
    211-220``, and its unbuilt ``StreamingBuffer``, ``tasks.md:362-368``).

    A chunk of ``chunk_frames`` new frames is emitted once ``context`` future frames
    exist; it is computed from the frames ``[start - context, end + context)`` and
    cropped (``context`` defaults to ``gen.receptive_field_frames()``, beyond which an
    output sample does not depend on the input: no overlap-add or crossfade is needed).
    Every chunk is bitwise the crop of ``gen(window)``.  In the exact-arithmetic modes
    (fp32, bf16x3) the concatenated stream is therefore BITWISE the one-shot
    ``gen(full_mel)``; in f16x3 each launch scales its operands by a power of two from
    the max over the item it sees — the window here, the whole utterance one-shot — and
    values whose f16 lo half falls below the normal range (< 2^-17 of that max) round on a
    different grid, so the stream equals the one-shot run to ~1e-8 at default scale (tested
    <= 1e-7) and is as accurate as it at any scale (2x weights: 4.8e-7 apart, both 1.65e-6 from
    the reference); both within 1e-4 of the reference.  Needs an exact-upsampling config (out = T x hop).

    Bounded state: a stream keeps only the frames ``[emitted - context, received)``.  Each
    stream owns one fixed buffer whose live columns start at a moving offset: a step only
    advances the offset past frames no later chunk reads (no copy), and the live columns
    move back to the front only when a feed would run past the end (amortised over several
    chunks), so memory and per-step cost do not grow with the stream's length.

    Several streams (``n_streams``) share each forward: :meth:`feed` appends frames
    without computing, :meth:`step` vocodes the next ready chunk of EVERY stream as one
    ragged batch (per-item lengths, ``hfg_forward_ex``; each item equals its window
    run alone, so batching changes no sample; the batch is gathered from the stream
    buffers in one copy), :meth:`finish` marks a stream's end so its tail is emitted by
    the following steps.  :meth:`push` / :meth:`flush` are the one-stream convenience
    (feed, then step until nothing is ready).  With ``debug_shapes`` (default: the
    generator's, i.e. ``DEBUG_SHAPES=1``) every chunk prints its shapes (Requirement 18.4).
    """

    def __init__(self, gen, chunk_frames: int = 64, context: Optional[int] = None,
                 n_streams: int = 1, debug_shapes: Optional[bool] = None):
        self.gen = gen
        self.hop = gen.output_length(2) - gen.output_length(1)
        if gen.output_length(7) != 7 * self.hop:
            raise ValueError("streaming needs exact upsampling (out_len = T * hop)")
        if chunk_frames < 1 or n_streams < 1:
            raise ValueError("chunk_frames and n_streams must be >= 1")
        self.chunk = int(chunk_frames)
        self.ctx = int(context) if context is not None else gen.receptive_field_frames()
        self.n_streams = int(n_streams)
        self.debug_shapes = (getattr(gen, "debug_shapes", False) if debug_shapes is None
                             else bool(debug_shapes))
        # widest window a step reads; a gathered window may run past a stream's live
        # columns by up to this much (read, never used: the forward masks by length)
        self._wmax = self.chunk + 2 * self.ctx
        self._buf: List[Optional[torch.Tensor]] = [None] * self.n_streams  # [n_mels, cap]
        self._pos = [0] * self.n_streams       # buffer column of frame _start
        self._start = [0] * self.n_streams     # absolute frame index of the first live column
        self._fill = [0] * self.n_streams      # live columns
        self._done = [False] * self.n_streams
        self._emitted = [0] * self.n_streams   # frames whose audio was returned
        self.chunks_run = 0
        self.compactions = 0
        self.last_windows: Dict[int, tuple] = {}  # stream -> (a, b, lo, hi) of the last step

    # -- state -------------------------------------------------------------------------
    @property
    def emitted(self) -> int:
        return self._emitted[0]

    def received(self, stream: int = 0) -> int:
        return self._start[stream] + self._fill[stream]

    def buffered_frames(self, stream: int = 0) -> int:
        """Frames currently held for `stream` (bounded: <= chunk + 2 context + a push)."""
        return self._fill[stream]

    def capacity(self, stream: int = 0) -> int:
        b = self._buf[stream]
        return 0 if b is None else b.shape[1]

    def feed(self, frames: torch.Tensor, stream: int = 0) -> None:
        """Append mel frames [n_mels, t] (or [1, n_mels, t]) to `stream`; no compute."""
        if frames.dim() == 3:
            frames = frames[0]
        if self._done[stream]:
            raise RuntimeError(f"stream {stream} was finished")
        t = frames.shape[1]
        if t == 0:
            return
        buf, pos, fill = self._buf[stream], self._pos[stream], self._fill[stream]
        # invariant after a feed: pos + fill + wmax <= cap (a step's gather stays in bounds)
        if buf is None or buf.device != frames.device or pos + fill + t + self._wmax > buf.shape[1]:
            if (buf is not None and buf.device == frames.device
                    and fill + t + self._wmax <= buf.shape[1]):
                if fill:  # live columns back to the front; overlapping ranges: clone first
                    src = buf[:, pos:pos + fill]
                    buf[:, :fill].copy_(src.clone() if fill > pos else src)
                self.compactions += 1
            else:
                # room for a few chunks of slack: a compaction every ~2 chunks at most
                cap = 2 * (self.chunk + 2 * self.ctx + t) + self._wmax + fill
                nb = torch.zeros(frames.shape[0], cap, dtype=torch.float32, device=frames.device)
                if buf is not None and fill:
                    nb[:, :fill].copy_(buf[:, pos:pos + fill])
                self._buf[stream] = buf = nb
            self._pos[stream] = pos = 0
        buf[:, pos + fill:pos + fill + t].copy_(frames)
        self._fill[stream] = fill + t

    def finish(self, stream: int = 0) -> None:
        """No more frames for `stream`: its remaining audio is emitted by later steps."""
        self._done[stream] = True

    def _window(self, s: int):
        """(a, b, lo, hi) absolute frames of `s`'s next ready chunk, or None."""
        T, a = self.received(s), self._emitted[s]
        if self._done[s]:
            if a >= T:
                return None
            b = min(T, a + self.chunk)
        else:
            if T - a < self.chunk + self.ctx:
                return None
            b = a + self.chunk
        return a, b, max(0, a - self.ctx), min(T, b + self.ctx)

    def _trim(self, s: int) -> None:
        """Drop frames no future chunk reads (keep [emitted - ctx, received)): the live
        range's offset moves, nothing is copied."""
        keep_from = max(self._start[s], self._emitted[s] - self.ctx)
        drop = keep_from - self._start[s]
        if drop > 0:
            self._pos[s] += drop
            self._start[s] = keep_from
            self._fill[s] -= drop

    def step(self, streams: Optional[Sequence[int]] = None) -> Dict[int, torch.Tensor]:
        """One batched forward over every stream (of `streams`, default all) with a ready
        chunk -> {stream: audio of that chunk}."""
        cand = range(self.n_streams) if streams is None else streams
        ready = [(s, w) for s in cand if (w := self._window(s)) is not None]
        if not ready:
            return {}
        lens = [hi - lo for _, (a, b, lo, hi) in ready]
        W = max(lens)
        # one gather (a batched copy of the strided windows); columns past an item's length
        # are whatever the buffer holds there: the forward reads a ragged item only below
        # its length
        views = [self._buf[s][:, self._pos[s] + lo - self._start[s]:
                              self._pos[s] + lo - self._start[s] + W]
                 for s, (a, b, lo, hi) in ready]
        mel = torch.stack(views)
        with torch.no_grad():
            wav = self.gen(mel, lengths=None if min(lens) == W else lens)
        out = {}
        self.last_windows = {s: w for s, w in ready}
        for i, (s, (a, b, lo, hi)) in enumerate(ready):
            out[s] = wav[i, 0, (a - lo) * self.hop:(b - lo) * self.hop]
            if self.debug_shapes:
                print(f"[StreamingVocoder] stream {s} chunk {self.chunks_run}: frames [{a}, {b}) "
                      f"context [{lo}, {hi}) mel {tuple(mel[i:i + 1, :, :hi - lo].shape)} -> "
                      f"wav {tuple(out[s].shape)}")
            self._emitted[s] = b
            self._trim(s)
        self.chunks_run += 1
        return out

    def push(self, frames: torch.Tensor, stream: int = 0) -> torch.Tensor:
        """Feed `frames` to `stream` and return all of its audio that is final now."""
        self.feed(frames, stream)
        return self._drain(stream)

    def flush(self, stream: int = 0) -> torch.Tensor:
        """End `stream` and return the rest of its audio."""
        self.finish(stream)
        return self._drain(stream)

    def _drain(self, stream: int) -> torch.Tensor:
        out = []
        while self._window(stream) is not None:
            out.append(self.step([stream])[stream])
        if out:
            return torch.cat(out)
        b = self._buf[stream]
        return torch.zeros(0, device=b.device if b is not None else None)
