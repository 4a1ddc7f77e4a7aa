"""Drop-in HiFi-GAN Generator for MI355X: the host-side mirror of the reference
interface, running on the HIP kernels of libhifigan_hip.so.

Mirrors ``models/hifigan.py`` of terrense/TTS-sambert_hifiGAN:

* ``get_padding``          models/hifigan.py:21-23
* ``ResBlock``             models/hifigan.py:26-86   (parameter container)
* ``MRF``                  models/hifigan.py:89-131  (parameter container)
* ``HiFiGANGenerator``     models/hifigan.py:134-283 (same ctor signature, same
                           submodule tree ⇒ identical state_dict keys, same
                           ``debug_shapes`` / ``DEBUG_SHAPES`` printing, same
                           ``apply_weight_norm`` / ``remove_weight_norm``)
* ``HiFiGAN``              models/hifigan.py:618-800, generation half
                           (``forward`` / ``generate``); ``discriminate`` is
                           GAN training and out of scope.

``HiFiGANGenerator.forward`` hands ``mel.data_ptr()``, a workspace from torch's
caching allocator and torch's current HIP stream to ``hfg_forward_ws``; the 78
kernel launches run asynchronously on that stream.  The parameters live in the
usual ``nn.Conv1d`` / ``nn.ConvTranspose1d`` containers (so ``state_dict`` /
``load_state_dict`` are unchanged) and are re-packed into the kernels' layout
whenever any of them changes.  Inference only: there is no CPU fallback and no
autograd; a CPU input or an input that requires grad raises.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib


def _lengths_on(lengths, device) -> torch.Tensor:
    """Per-item lengths as a contiguous int32 tensor on `device`.  A host list goes through
    pinned memory with a non-blocking copy: a pageable host-to-device copy would make the
    host wait for all work already queued on the stream (every ragged forward a sync)."""
    if isinstance(lengths, torch.Tensor) and lengths.device == device:
        return lengths.to(torch.int32).contiguous()
    host = torch.as_tensor(lengths).to(torch.int32).contiguous()
    if host.device.type == "cpu":
        host = host.pin_memory()
    return host.to(device, non_blocking=True)


PRECISIONS = ("f16x3", "fp32", "bf16x3", "bf16w")


def default_precision() -> str:
    """The precision a module gets when its constructor is not given one: "f16x3"
    (fp32-class split products on the f16 matrix cores, include/hifigan_hip.h), or
    ``HFG_PRECISION`` from the environment ("f16x3", "fp32", "bf16x3", "bf16w"), so a
    reference code base can switch its Generator's arithmetic without code changes."""
    p = os.environ.get("HFG_PRECISION", "f16x3")
    if p not in PRECISIONS:
        raise ValueError(f"HFG_PRECISION={p!r}: expected one of {', '.join(PRECISIONS)}")
    return p


def get_padding(kernel_size: int, dilation: int = 1) -> int:
    """Calculate padding to maintain sequence length (models/hifigan.py:21-23)."""
    return int((kernel_size * dilation - dilation) / 2)


class _HipWeights(nn.Module):
    """Weight tracking shared by the modules that run on a C-ABI handle.

    The parameters stay in ordinary ``nn.Conv1d`` / ``nn.ConvTranspose1d``
    containers; a handle per device holds them packed in the kernels' layout.  They
    are re-packed before a forward when any parameter was replaced, resized or
    moved (data_ptr / shape), bumped its autograd version (in-place ops, ``copy_``
    under no_grad), and after ``load_state_dict`` / ``.to()`` / ``refresh_weights()``.
    The check is host-side bookkeeping only: a forward launches asynchronously, with
    no host sync.  An edit through ``param.data`` leaves the version counter untouched:
    call ``refresh_weights()`` after one, or set ``verify_weights = True`` (opt-in) to
    compare a device-side content hash of the parameters (``hfg_checksum32``) before
    every forward — one small D2H read, i.e. a stream sync per forward (skipped while a
    hipGraph is being captured).
    """

    verify_weights = False

    def _hip_setup(self, precision: Optional[str]):
        precision = default_precision() if precision is None else precision
        self._hfg_handles: Dict[int, _lib.Handle] = {}
        self._hfg_fingerprint: Dict[int, tuple] = {}
        self._hfg_checksum: Dict[int, torch.Tensor] = {}
        self._hfg_items = None  # cached (key, tensor) list, rebuilt after any invalidation
        self._hfg_slots = []    # (conv, parameter name, tensor) the cache was built from
        self.precision = precision
        self.register_load_state_dict_post_hook(_HipWeights._after_load)

    @staticmethod
    def _after_load(module, _incompatible_keys) -> None:
        # torch requires load_state_dict post hooks to return None
        module.refresh_weights()

    def refresh_weights(self):
        """Force a re-pack of the parameters before the next forward."""
        self._hfg_fingerprint = {}
        self._hfg_checksum = {}
        self._hfg_items = None
        return self

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self.refresh_weights()  # a shared submodule moved elsewhere shows in data_ptr
        return out

    def _items(self):
        """The (key, tensor) list, cached: walking the module tree costs ~0.6 ms for V1,
        more than a C1 forward's host budget.  Every forward checks that each cached tensor
        is still the one its conv holds (one dict lookup per parameter, ~15 us for V1), so a
        parameter replaced on any conv (``conv.weight = Parameter(..)``, weight norm applied
        or removed) rebuilds the list — no process-wide hook is installed."""
        items = self._hfg_items
        if items is not None and any(m._parameters.get(p) is not t
                                     for m, p, t in self._hfg_slots):
            items = None
        if items is None:
            items, slots = [], []
            for key, mod, p in self._hip_weight_slots():
                t = getattr(mod, p)
                items.append((key, t))
                if p in mod._parameters:
                    slots.append((mod, p, t))
            self._hfg_items, self._hfg_slots = items, slots
        return items

    # subclasses: (key, module, parameter name) of every parameter in the handle's key
    # space, and the handle
    def _hip_weight_slots(self):
        raise NotImplementedError

    def _hip_weight_items(self):
        return [(key, getattr(mod, p)) for key, mod, p in self._hip_weight_slots()]

    def _hip_new_handle(self, idx: int) -> _lib.Handle:
        raise NotImplementedError

    def _handle_for(self, device: torch.device) -> _lib.Handle:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        h = self._hfg_handles.get(idx)
        if h is None:
            h = self._hip_new_handle(idx)
            self._hfg_handles[idx] = h
        items = self._items()
        # in-place edits bump _version; replaced storage changes data_ptr (shapes and
        # devices only change with a new storage); one pass, ~50 us for V1's 156 tensors
        fp = (tuple([t._version for _, t in items]), tuple([t.data_ptr() for _, t in items]))
        stale = self._hfg_fingerprint.get(idx) != fp
        check = self.verify_weights and not torch.cuda.is_current_stream_capturing()
        dev_ts = ([t.detach() for _, t in items if t.is_cuda and t.dtype == torch.float32
                   and t.is_contiguous()] if check else [])
        check = check and bool(dev_ts)
        cks = None
        if not stale and check:
            cks = _lib.checksum32(dev_ts)
            stale = not torch.equal(cks, self._hfg_checksum.get(idx, torch.empty(0)))
        if stale:
            for k, t in items:
                h.set_weight(k, t)
            h.commit()
            self._hfg_fingerprint[idx] = fp
            if check:
                self._hfg_checksum[idx] = cks if cks is not None else _lib.checksum32(dev_ts)
        return h

    @staticmethod
    def _conv_slots(module: nn.Module, prefix: str = ""):
        for name, mod in module.named_modules():
            if not isinstance(mod, (nn.Conv1d, nn.ConvTranspose1d)):
                continue
            names = (("weight_g", "weight_v") if hasattr(mod, "weight_g") and hasattr(mod, "weight_v")
                     else ("weight",))
            for p in names + ("bias",):
                yield prefix + name + "." + p, mod, p

    def _run_block(self, x: torch.Tensor, channels: int, resblock: int) -> torch.Tensor:
        """y = MRF(x) (resblock < 0) or ResBlock_resblock(x) on the HIP device."""
        if not isinstance(x, torch.Tensor) or x.dim() != 3 or x.shape[1] != channels:
            raise RuntimeError(f"expected x [B, {channels}, T], got {getattr(x, 'shape', type(x))}")
        if not x.is_cuda:
            raise RuntimeError("the MI355X ResBlock / MRF run on the HIP device only; move x to "
                               "'cuda' (there is no CPU fallback)")
        if torch.is_grad_enabled() and x.requires_grad:
            raise NotImplementedError("inference-only HIP path: no autograd")
        B, _, L = x.shape
        if B == 0 or L == 0:
            raise RuntimeError("empty input")
        xc = x.detach().to(torch.float32).contiguous()
        with torch.cuda.device(x.device):
            h = self._handle_for(x.device)
            y = torch.empty_like(xc)
            ws_bytes = h.mrf_workspace_bytes(B, L)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
            h.mrf_forward(xc.data_ptr(), B, L, y.data_ptr(), ws.data_ptr(), ws_bytes,
                          torch.cuda.current_stream(x.device).cuda_stream, resblock=resblock)
        return y


class ResBlock(_HipWeights):
    """ResBlock (models/hifigan.py:26-86): ``convs1[m]`` = Conv1d(C, C, k, dilation=d_m),
    ``convs2[m]`` = Conv1d(C, C, k); forward = for each m: x += conv2(lrelu(conv1(lrelu(x)))).
    Inside a Generator its computation is part of the fused schedule; called on its own
    it runs ``hfg_resblock_forward`` on an MRF handle of this one block."""

    def __init__(self, channels: int, kernel_size: int = 3, dilation: Tuple[int, ...] = (1, 3, 5),
                 *, precision: Optional[str] = None):
        super().__init__()
        self.channels = channels
        self.kernel_size = kernel_size
        self.dilation = tuple(dilation)
        self.convs1 = nn.ModuleList()
        self.convs2 = nn.ModuleList()
        for d in dilation:
            self.convs1.append(nn.Conv1d(channels, channels, kernel_size, stride=1, dilation=d,
                                         padding=get_padding(kernel_size, d)))
            self.convs2.append(nn.Conv1d(channels, channels, kernel_size, stride=1, dilation=1,
                                         padding=get_padding(kernel_size, 1)))
        self._hip_setup(precision)

    def _hip_weight_slots(self):
        return self._conv_slots(self, "resblocks.0.")

    def _hip_new_handle(self, idx):
        cfg = _lib.make_mrf_config(self.channels, [self.kernel_size], [list(self.dilation)],
                                   precision=self.precision)
        return _lib.Handle(cfg, idx, mrf=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, C, T] -> [B, C, T] (models/hifigan.py:72-86)."""
        if not self.dilation:
            return x
        return self._run_block(x, self.channels, 0)


class MRF(_HipWeights):
    """Multi-Receptive Field module (models/hifigan.py:89-131): the mean of its
    ResBlocks' outputs on the same input.  Called on its own it runs
    ``hfg_mrf_forward`` on an MRF handle with this module's state_dict keys."""

    def __init__(self, channels: int, resblock_kernel_sizes: List[int] = [3, 7, 11],
                 resblock_dilation_sizes: List[List[int]] = [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                 *, precision: Optional[str] = None):
        super().__init__()
        precision = default_precision() if precision is None else precision
        self.channels = channels
        self.resblock_kernel_sizes = list(resblock_kernel_sizes)
        self.resblock_dilation_sizes = [list(d) for d in resblock_dilation_sizes]
        self.resblocks = nn.ModuleList()
        for kernel_size, dilations in zip(resblock_kernel_sizes, resblock_dilation_sizes):
            self.resblocks.append(ResBlock(channels, kernel_size, tuple(dilations),
                                           precision=precision))
        self._hip_setup(precision)

    def _hip_weight_slots(self):
        return self._conv_slots(self)

    def _hip_new_handle(self, idx):
        cfg = _lib.make_mrf_config(self.channels, self.resblock_kernel_sizes,
                                   self.resblock_dilation_sizes, precision=self.precision)
        return _lib.Handle(cfg, idx, mrf=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, C, T] -> mean_j ResBlock_j(x) [B, C, T] (models/hifigan.py:116-131)."""
        return self._run_block(x, self.channels, -1)


class HiFiGANGenerator(_HipWeights):
    """HiFi-GAN Generator, mel [B, n_mels, Tfrm] → wav [B, 1, T_wav] on MI355X.

    Same constructor as models/hifigan.py:149-158.
    """

    def __init__(
        self,
        n_mels: int = 80,
        upsample_rates: List[int] = [8, 8, 2, 2],
        upsample_kernel_sizes: List[int] = [16, 16, 4, 4],
        upsample_initial_channel: int = 512,
        resblock_kernel_sizes: List[int] = [3, 7, 11],
        resblock_dilation_sizes: List[List[int]] = [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
        debug_shapes: bool = False,
        *,
        precision: Optional[str] = None,
    ):
        super().__init__()
        precision = default_precision() if precision is None else precision
        self.n_mels = n_mels
        self.num_kernels = len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_rates)
        self.debug_shapes = debug_shapes or os.getenv("DEBUG_SHAPES", "0") == "1"

        self.conv_pre = nn.Conv1d(n_mels, upsample_initial_channel, kernel_size=7, stride=1,
                                  padding=3)
        self.ups = nn.ModuleList()
        self.mrfs = nn.ModuleList()
        for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
            in_channels = upsample_initial_channel // (2 ** i)
            out_channels = upsample_initial_channel // (2 ** (i + 1))
            self.ups.append(nn.ConvTranspose1d(in_channels, out_channels, kernel_size=k, stride=u,
                                               padding=(k - u) // 2))
            self.mrfs.append(MRF(out_channels, resblock_kernel_sizes, resblock_dilation_sizes,
                                 precision=precision))
        final_channels = upsample_initial_channel // (2 ** self.num_upsamples)
        self.conv_post = nn.Conv1d(final_channels, 1, kernel_size=7, stride=1, padding=3)

        self._hfg_args = (n_mels, upsample_rates, upsample_kernel_sizes, upsample_initial_channel,
                          resblock_kernel_sizes, resblock_dilation_sizes)
        self._hip_setup(precision)
        self.set_precision(self.precision)

    def set_precision(self, precision: str):
        """"f16x3" (the module default, ``default_precision``: fp32 operands scaled by a
        power of two and split into two f16 halves on the f16 matrix cores, fp32-class
        products), "fp32" (exact fp32 MFMA; the C ABI's zero-initialised default),
        "bf16x3" (two bf16 halves; within ~1e-5 of the reference at default weight scale) or "bf16w" (conv weights stored as bf16 — rounded when
        committed to the handle, the module's own parameters untouched — activations
        still split: the reference model with bf16-cast weights, to 1e-4).  Applies to
        the MRF / ResBlock submodules too."""
        self._hfg_cfg = _lib.make_config(*self._hfg_args, precision=precision)
        for m in self.modules():
            if isinstance(m, _HipWeights):
                m.precision = precision
                m._hfg_handles = {}
                m.refresh_weights()
        return self

    # ------------------------------------------------------------------
    def _hip_weight_slots(self):
        """(state_dict-style key, conv, name) of every parameter the kernels need,
        with weight_g / weight_v passed through for weight-normed modules."""
        return self._conv_slots(self)

    def _weight_tensors(self):
        return self._hip_weight_items()

    def _hip_new_handle(self, idx):
        return _lib.Handle(self._hfg_cfg, idx)

    def hip_handle(self, device=None) -> _lib.Handle:
        """The C-ABI handle for ``device`` with the current weights committed."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        return self._handle_for(torch.device(device))

    def output_length(self, t: int) -> int:
        length = t
        for u, k in zip(self._hfg_cfg.up_rates[: self.num_upsamples],
                        self._hfg_cfg.up_kernels[: self.num_upsamples]):
            length = (length - 1) * u - 2 * ((k - u) // 2) + k
        return length

    # ------------------------------------------------------------------
    def forward(self, mel: torch.Tensor, *, lengths=None, mel_layout: str = "bct") -> torch.Tensor:
        """Generate waveform from mel-spectrogram (models/hifigan.py:224-261).

        Args:
            mel: [B, n_mels, Tfrm] float32 on a HIP device ([B, Tfrm, n_mels] with
                 ``mel_layout="btc"``, the acoustic model's output layout).
            lengths: optional valid frames per utterance of a zero-padded batch
                 (sequence of ints or an int tensor).  Item b's wav then equals the
                 Generator run on mel[b, :, :lengths[b]] alone, zero past
                 ``output_length(lengths[b])``.
        Returns:
            wav: [B, 1, T_wav] float32, T_wav = Tfrm * prod(upsample_rates)
        """
        if self.debug_shapes:
            print(f"[HiFiGANGenerator] Input mel shape: {mel.shape}")
        if not isinstance(mel, torch.Tensor) or mel.dim() != 3:
            raise RuntimeError(f"expected mel [B, n_mels, T], got {getattr(mel, 'shape', type(mel))}")
        if mel_layout not in ("bct", "btc"):
            raise ValueError("mel_layout must be 'bct' or 'btc'")
        n_ch = mel.shape[1] if mel_layout == "bct" else mel.shape[2]
        if n_ch != self.n_mels:
            raise RuntimeError(f"expected {self.n_mels} mel channels, got {n_ch}")
        if not mel.is_cuda:
            raise RuntimeError("HiFiGANGenerator (MI355X) runs on the HIP device only; "
                               "move the mel to 'cuda' (there is no CPU fallback)")
        if torch.is_grad_enabled() and mel.requires_grad:
            raise NotImplementedError("inference-only HIP path: no autograd through the Generator")
        B = mel.shape[0]
        T = mel.shape[2] if mel_layout == "bct" else mel.shape[1]
        if B == 0 or T == 0:
            raise RuntimeError("empty mel input")
        mel_c = mel.detach().to(torch.float32).contiguous()
        with torch.cuda.device(mel.device):
            h = self._handle_for(mel.device)
            out_len = h.out_len(T)
            wav = torch.empty((B, 1, out_len), dtype=torch.float32, device=mel.device)
            ws_bytes = h.workspace_bytes(B, T)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=mel.device)
            stream = torch.cuda.current_stream(mel.device).cuda_stream
            if lengths is None and mel_layout == "bct":
                h.forward_ws(mel_c.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(),
                             ws_bytes, stream)
            else:
                lens_t = None
                if lengths is not None:
                    lens_t = _lengths_on(lengths, mel.device)
                    if lens_t.shape != (B,):
                        raise RuntimeError(f"lengths must have shape [{B}]")
                h.forward_ex(mel_c.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(),
                             ws_bytes, stream, mel_layout=mel_layout,
                             lengths_ptr=lens_t.data_ptr() if lens_t is not None else 0)
        if self.debug_shapes:
            x_len = T
            c = self.conv_pre.out_channels
            print(f"[HiFiGANGenerator] After conv_pre: {torch.Size([B, c, x_len])}")
            for i, up in enumerate(self.ups):
                u, k = up.stride[0], up.kernel_size[0]
                x_len = (x_len - 1) * u - 2 * ((k - u) // 2) + k
                c = up.out_channels
                print(f"[HiFiGANGenerator] After upsample {i}: {torch.Size([B, c, x_len])}")
                print(f"[HiFiGANGenerator] After MRF {i}: {torch.Size([B, c, x_len])}")
            print(f"[HiFiGANGenerator] Output wav shape: {wav.shape}")
        return wav

    def forward_with_stages(self, mel: torch.Tensor):
        """(wav, {stage: tensor}) — the forward (one stream) plus copies of the tensors the
        reference's forward passes through (models/hifigan.py:238-251): "conv_pre",
        "ups.i" (after each ConvTranspose1d) and "mrfs.i" (after each MRF).  Inspection
        entry hfg_forward_taps (include/hifigan_hip_inspect.h); for parity checks."""
        if not (isinstance(mel, torch.Tensor) and mel.dim() == 3 and mel.is_cuda):
            raise RuntimeError("expected a HIP mel [B, n_mels, T]")
        B, _, T = mel.shape
        mel_c = mel.detach().to(torch.float32).contiguous()
        with torch.cuda.device(mel.device):
            h = self._handle_for(mel.device)
            out_len = h.out_len(T)
            wav = torch.empty((B, 1, out_len), dtype=torch.float32, device=mel.device)
            stages = {"conv_pre": torch.empty(B, self.conv_pre.out_channels, T, device=mel.device)}
            x_len = T
            for i, up in enumerate(self.ups):
                u, k = up.stride[0], up.kernel_size[0]
                x_len = (x_len - 1) * u - 2 * ((k - u) // 2) + k
                for name in (f"ups.{i}", f"mrfs.{i}"):
                    stages[name] = torch.empty(B, up.out_channels, x_len, device=mel.device)
            ws_bytes = h.workspace_bytes(B, T)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=mel.device)
            h.forward_taps(mel_c.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(),
                           ws_bytes, [t.data_ptr() for t in stages.values()],
                           torch.cuda.current_stream(mel.device).cuda_stream)
        return wav, stages

    def receptive_field_frames(self) -> int:
        """Upper bound, in mel frames, of how far (each side) an output sample's
        value depends on the input: conv_pre + per-stage upsampler and MRF halos
        + conv_post, each divided by the stage's samples-per-frame.  A chunk with
        this many context frames on both sides reproduces the full-length run."""
        rate = 1
        halo = 3.0  # conv_pre k=7
        for up, mrf in zip(self.ups, self.mrfs):
            u, k = up.stride[0], up.kernel_size[0]
            halo += -(-k // u) / rate  # taps per output phase, in input samples
            rate *= u
            best = 0
            for rb in mrf.resblocks:
                s = 0
                for c1, c2 in zip(rb.convs1, rb.convs2):
                    s += c1.padding[0] + c2.padding[0]
                best = max(best, s)
            halo += best / rate
        halo += 3.0 / rate  # conv_post k=7
        return int(halo) + 1

    def remove_weight_norm(self):
        """models/hifigan.py:263-272"""
        for layer in self.ups:
            nn.utils.remove_weight_norm(layer)
        for mrf in self.mrfs:
            for resblock in mrf.resblocks:
                for conv in resblock.convs1:
                    nn.utils.remove_weight_norm(conv)
                for conv in resblock.convs2:
                    nn.utils.remove_weight_norm(conv)

    def apply_weight_norm(self):
        """models/hifigan.py:274-283 (the kernels fold g·v/||v|| at commit)."""
        for layer in self.ups:
            nn.utils.weight_norm(layer)
        for mrf in self.mrfs:
            for resblock in mrf.resblocks:
                for conv in resblock.convs1:
                    nn.utils.weight_norm(conv)
                for conv in resblock.convs2:
                    nn.utils.weight_norm(conv)


class HiFiGAN(nn.Module):
    """Generation half of the reference ``HiFiGAN`` wrapper (models/hifigan.py:618-800).

    Accepts the reference constructor arguments; the discriminator arguments
    are accepted and ignored because ``discriminate`` (GAN training) is out of
    scope for this inference path.
    """

    def __init__(self, n_mels: int = 80, upsample_rates: List[int] = [8, 8, 2, 2],
                 upsample_kernel_sizes: List[int] = [16, 16, 4, 4],
                 upsample_initial_channel: int = 512,
                 resblock_kernel_sizes: List[int] = [3, 7, 11],
                 resblock_dilation_sizes: List[List[int]] = [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                 msd_use_spectral_norm: bool = False, mpd_periods: List[int] = [2, 3, 5, 7, 11],
                 mpd_use_spectral_norm: bool = False, debug_shapes: bool = False, *,
                 precision: Optional[str] = None):
        super().__init__()
        self.debug_shapes = debug_shapes or os.getenv("DEBUG_SHAPES", "0") == "1"
        self.generator = HiFiGANGenerator(
            n_mels=n_mels, upsample_rates=upsample_rates,
            upsample_kernel_sizes=upsample_kernel_sizes,
            upsample_initial_channel=upsample_initial_channel,
            resblock_kernel_sizes=resblock_kernel_sizes,
            resblock_dilation_sizes=resblock_dilation_sizes, debug_shapes=debug_shapes,
            precision=precision)
        self.msd = None
        self.mpd = None

    def forward(self, mel: torch.Tensor) -> torch.Tensor:
        """models/hifigan.py:704-724"""
        if self.debug_shapes:
            print(f"[HiFiGAN] forward() - Input mel shape: {mel.shape}")
        wav = self.generator(mel)
        if self.debug_shapes:
            print(f"[HiFiGAN] forward() - Output wav shape: {wav.shape}")
        return wav

    def generate(self, mel: torch.Tensor) -> torch.Tensor:
        """models/hifigan.py:790-800"""
        return self.forward(mel)

    def discriminate(self, wav_real, wav_fake):
        raise NotImplementedError("discriminators are GAN-training only; out of scope for the "
                                  "MI355X inference path")

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Accepts a full reference HiFiGAN state_dict: msd.* / mpd.* keys are dropped."""
        sd = {k: v for k, v in state_dict.items() if not k.startswith(("msd.", "mpd."))}
        return super().load_state_dict(sd, strict=strict, assign=assign)
