"""Host logic of the streaming vocoder (glue.StreamingVocoder) on CPU with a stand-in
generator of finite receptive field: chunk windows, bounded buffers, multi-stream
batching through per-item lengths, the finish/flush tail and the per-chunk shape lines.
Integer-valued mels keep every sum exact, so "equal to the one-shot run" is bitwise
here as it is on the GPU (tests/test_gpu_glue.py)."""
import importlib

import numpy as np
import torch


class _Fake:
    """Per-utterance 7-tap filter of the channel sum, hop 4, zero past each length:
    receptive field 3 frames each side, like a tiny Generator."""
    debug_shapes = False

    def __init__(self):
        self.calls = []  # batch size of every forward

    def output_length(self, t):
        return 4 * int(t)

    def receptive_field_frames(self):
        return 3

    def __call__(self, mel, lengths=None, mel_layout="bct"):
        B, C, T = mel.shape
        self.calls.append(B)
        lens = [T] * B if lengths is None else list(lengths)
        out = torch.zeros(B, 1, 4 * T)
        for b in range(B):
            x = torch.nn.functional.pad(mel[b, :, :lens[b]].sum(0), (3, 3))
            y = sum(x[k:k + lens[b]] * (k + 1) for k in range(7))
            out[b, 0, :4 * lens[b]] = y.repeat_interleave(4)
        return out


def _glue(pkg):
    return importlib.import_module("tts_sambert_hifigan_amd.glue")


def _mels(lengths, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(-8, 9, (5, n), generator=g).float() for n in lengths]


def test_multi_stream_batched_equals_one_shot_and_is_bounded(pkg):
    glue, gen = _glue(pkg), _Fake()
    mels = _mels((100, 37, 1, 64, 9))
    ref = [gen(m[None])[0, 0] for m in mels]
    S, chunk = len(mels), 8
    sv = glue.StreamingVocoder(gen, chunk_frames=chunk, n_streams=S)
    outs = {s: [] for s in range(S)}
    pos = [0] * S
    rng = np.random.default_rng(1)
    gen.calls.clear()
    while any(pos[s] < mels[s].shape[1] for s in range(S)):
        for s in range(S):
            if pos[s] < mels[s].shape[1]:
                n = int(rng.integers(1, 10))
                sv.feed(mels[s][:, pos[s]:pos[s] + n], s)
                pos[s] += n
                if pos[s] >= mels[s].shape[1]:
                    sv.finish(s)
        for s, a in sv.step().items():
            outs[s].append(a)
        assert max(sv.buffered_frames(s) for s in range(S)) <= chunk + 2 * 3 + 9
    while True:
        r = sv.step()
        if not r:
            break
        for s, a in r.items():
            outs[s].append(a)
    for s in range(S):
        assert torch.equal(torch.cat(outs[s]), ref[s]), s
    assert max(gen.calls) > 1  # streams really shared forwards
    # fixed per-stream buffers: live columns + slack for the gather and a few chunks
    w = chunk + 2 * 3
    assert max(sv.capacity(s) for s in range(S)) <= 2 * (w + 9) + w + (w + 9)


def test_single_stream_push_flush_constant_state(pkg, capsys):
    glue, gen = _glue(pkg), _Fake()
    mel = _mels((2000,), seed=3)[0]
    ref = gen(mel[None])[0, 0]
    sv = glue.StreamingVocoder(gen, chunk_frames=16, debug_shapes=True)
    pieces, caps = [], set()
    for i in range(0, 2000, 7):
        pieces.append(sv.push(mel[:, i:i + 7]))
        caps.add(sv.capacity())
        assert sv.buffered_frames() <= 16 + 2 * 3 + 7
    pieces.append(sv.flush())
    assert torch.equal(torch.cat(pieces), ref)
    assert len(caps) == 1  # one allocation for the whole stream
    # trimming moves an offset; the live columns are copied back to the front only
    # every few chunks
    assert 0 < sv.compactions <= sv.chunks_run // 2
    lines = [l for l in capsys.readouterr().out.splitlines() if l.startswith("[StreamingVocoder]")]
    assert len(lines) == sv.chunks_run == -(-2000 // 16)
    assert "mel (1, 5, " in lines[1] and "-> wav (64,)" in lines[1]
