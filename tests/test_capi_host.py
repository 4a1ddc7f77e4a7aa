"""C ABI on the CPU container: the library loads, exports every symbol the
headers declare, validates configurations, and packs weights into exactly the
GEMM layout the kernels consume (checked by a numpy emulation of the kernels'
implicit GEMM, incl. the polyphase ConvTranspose1d).  No compute call needs a
GPU: handles are host-only (device = -1)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT
from oracle import config as C

# kTiles of csrc/kernels.h: (WM, WN, WAVES_M, WAVES_N)
TILES = [(2, 2, 2, 2), (2, 2, 1, 4), (1, 4, 1, 4)]


def header_symbols():
    syms = set()
    for h in ("hifigan_hip.h", "hifigan_hip_inspect.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b(hfg_[a-z0-9_]+)\s*\(", src))
    return syms


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.load_library()
    syms = header_symbols()
    assert len(syms) == 43
    for s in sorted(syms):
        assert hasattr(lib, s), f"missing export {s}"
    assert set(syms) == set(pkg._lib.SIGNATURES), "ctypes signatures out of sync with headers"
    assert b"gfx950" in lib.hfg_version()


def host_handle(pkg, cfg, precision="fp32"):
    c = pkg.make_config(**{k: v for k, v in cfg.kwargs().items()}, precision=precision)
    return pkg.Handle(c, -1)


def test_create_validates_config(pkg):
    lib = pkg.load_library()
    c = pkg.make_config(80, [8, 8, 2, 2], [16, 16, 4, 4], 512, [3, 7, 11], [[1, 3, 5]] * 3)
    c.dtype = 7
    h = ctypes.c_void_p()
    assert lib.hfg_create(ctypes.byref(c), -1, ctypes.byref(h)) == -22
    assert b"dtype" in lib.hfg_last_error()
    c.dtype = 0
    c.up_rates[0] = 0
    assert lib.hfg_create(ctypes.byref(c), -1, ctypes.byref(h)) == -22
    assert lib.hfg_create(None, -1, ctypes.byref(h)) == -22


def test_out_len_and_workspace(pkg):
    for cfg in (C.V1, C.V2STAR, C.NONEXACT):
        h = host_handle(pkg, cfg)
        for t in (1, 17, 256):
            assert h.out_len(t) == C.out_len(cfg, t)
        assert h.workspace_bytes(8, 1024) >= 4 * 4 * 8 * 128 * 65536 * (cfg is C.V1)
    h = host_handle(pkg, C.V1)
    assert 0 <= h.workspace_bytes(8, 1024) - 4 * 4 * 8 * 128 * 65536 <= 4096
    assert pkg.load_library().hfg_num_params(h.ptr) == 156


def test_set_weight_errors_and_commit(pkg):
    h = host_handle(pkg, C.V2STAR)
    sd = C.make_state_dict(C.V2STAR, seed=3)
    with pytest.raises(pkg.HfgError) as e:
        h.set_weight("conv_pre.nope", torch.zeros(3))
    assert e.value.code == -22
    with pytest.raises(pkg.HfgError):
        h.set_weight("conv_pre.weight", torch.zeros(128, 80, 5))  # wrong k
    with pytest.raises(pkg.HfgError) as e:
        h.commit()  # nothing set yet
    assert e.value.code == -11
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    lib = pkg.load_library()
    rc = lib.hfg_forward(h.ptr, None, 1, 4, None, 1024, None)
    assert rc == -22  # host-only handle: no forward


def unpack_gemm(info, packed, cin):
    """Invert the fragment order of conv_kernels.hip → Wt[row][ci][j]."""
    WM, WN, WAVES_M, WAVES_N = TILES[info["tile"]]
    CK = info["CK"]
    MT = 32 * WM * WAVES_M
    assert MT == info["MT"]
    KK = CK // 2
    KT = info["KT"]
    shape = (info["m_tiles"], info["n_chunks"], KT, KK, WAVES_M, 64, WM)
    p = packed.reshape(shape)
    Wt = np.zeros((info["m_tiles"] * MT, info["n_chunks"] * CK, KT), np.float32)
    lane = np.arange(64)
    for mt in range(shape[0]):
        for c in range(shape[1]):
            for j in range(KT):
                for kk in range(KK):
                    for wv in range(WAVES_M):
                        for wm in range(WM):
                            rows = mt * MT + wv * 32 * WM + wm * 32 + (lane & 31)
                            cis = c * CK + 2 * kk + (lane >> 5)
                            Wt[rows, cis, j] = p[mt, c, j, kk, wv, :, wm]
    return Wt[: info["M"], :cin, :]


def emulate_conv(Wt, bias_rows, x, off, dil, N):
    """out[m][n] = bias[m] + sum_{ci,j} Wt[m][ci][j] * x[ci][n + off + j*dil] (zero padded)."""
    cin, L = x.shape
    M, _, KT = Wt.shape
    out = np.tile(bias_rows[:M, None].astype(np.float64), (1, N))
    for j in range(KT):
        idx = np.arange(N) + off + j * dil
        ok = (idx >= 0) & (idx < L)
        xs = np.zeros((cin, N))
        xs[:, ok] = x[:, idx[ok]]
        out += Wt[:, :, j].astype(np.float64) @ xs
    return out


@pytest.mark.parametrize("preset", ["v1", "v2star", "nonexact"])
def test_packing_emulates_conv_and_polyphase_upsample(pkg, preset):
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=21)
    h = host_handle(pkg, cfg)
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    rng = np.random.default_rng(0)
    c0 = cfg.upsample_initial_channel
    # every upsample layer: polyphase GEMM + scatter == F.conv_transpose1d
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cin, cout = c0 >> i, c0 >> (i + 1)
        info, packed, bias = pkg_layer(h, f"ups.{i}")
        assert info["kind"] == 1 and info["M"] == cout * u and info["KT"] == -(-k // u)
        Wt = unpack_gemm(info, packed, cin)
        Lin = 13
        x = rng.standard_normal((cin, Lin)).astype(np.float32)
        ref = F.conv_transpose1d(torch.from_numpy(x)[None], torch.from_numpy(sd[f"ups.{i}.weight"]),
                                 torch.from_numpy(sd[f"ups.{i}.bias"]), u, (k - u) // 2)[0].numpy()
        Lout = ref.shape[-1]
        p = (k - u) // 2
        N = (Lout - 1 + p) // u + 1
        g = emulate_conv(Wt, bias, x, -(info["KT"] - 1), 1, N)
        y = np.full((cout, Lout), np.nan)
        for m in range(cout * u):
            co, r = divmod(m, u)
            t = np.arange(N) * u + r - p
            ok = (t >= 0) & (t < Lout)
            y[co, t[ok]] = g[m, ok]
        assert not np.isnan(y).any()
        assert np.abs(y - ref).max() < 1e-4
    # one dilated ResBlock conv of each stage: GEMM == F.conv1d
    for i in range(len(cfg.upsample_rates)):
        ch = c0 >> (i + 1)
        kr, d = cfg.resblock_kernel_sizes[-1], cfg.resblock_dilation_sizes[-1][-1]
        mod = f"mrfs.{i}.resblocks.{len(cfg.resblock_kernel_sizes) - 1}.convs1.{len(cfg.resblock_dilation_sizes[-1]) - 1}"
        info, packed, bias = pkg_layer(h, mod)
        assert info["kind"] == 0 and info["M"] == ch and info["KT"] == kr
        Wt = unpack_gemm(info, packed, ch)
        x = rng.standard_normal((ch, 40)).astype(np.float32)
        pad = C.get_padding(kr, d)
        ref = F.conv1d(torch.from_numpy(x)[None], torch.from_numpy(sd[mod + ".weight"]),
                       torch.from_numpy(sd[mod + ".bias"]), 1, pad, d)[0].numpy()
        g = emulate_conv(Wt, bias, x, -pad, d, 40)
        assert np.abs(g - ref).max() < 1e-4


def pkg_layer(h, mod):
    return h.packed_layer(mod)


def test_weight_norm_fold(pkg):
    cfg = C.V2STAR
    wn = C.make_weight_norm_state_dict(cfg, seed=5)
    plain = {}
    for k, v in wn.items():
        if k.endswith("weight_g"):
            mod = k[:-9]
            vv = wn[mod + ".weight_v"].astype(np.float64)
            norm = np.sqrt((vv ** 2).reshape(vv.shape[0], -1).sum(1)).reshape(v.shape)
            plain[mod + ".weight"] = (v * vv / norm).astype(np.float32)
        elif not k.endswith("weight_v"):
            plain[k] = v
    h1, h2 = host_handle(pkg, cfg), host_handle(pkg, cfg)
    for k, v in wn.items():
        h1.set_weight(k, torch.from_numpy(v))
    for k, v in plain.items():
        h2.set_weight(k, torch.from_numpy(v))
    h1.commit()
    h2.commit()
    for mod in ("ups.1", "mrfs.2.resblocks.1.convs2.0", "conv_pre", "conv_post"):
        _, a, ab = h1.packed_layer(mod)
        _, b, bb = h2.packed_layer(mod)
        assert np.allclose(a, b, rtol=1e-6, atol=1e-7)
        assert np.array_equal(ab, bb)


def bf2f(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def h2f(u16):
    return np.ascontiguousarray(u16).view(np.float16).astype(np.float32)


def dec(u16, precision, ew=0):
    """A split plane's 16-bit values as float64: bf16 (bf16x3), or f16 halves of w * 2^ew
    (f16x3 / bf16w: csrc/bf16x3_common.h)."""
    if precision == "bf16x3":
        return bf2f(u16).astype(np.float64)
    return h2f(u16).astype(np.float64) * 2.0 ** -ew


# reconstruction bound of hi + lo relative to the layer's max |w|: bf16 halves ~2^-16, scaled
# f16 halves ~2^-22 (csrc/bf16x3_common.h)
SPLIT_TOL = {"bf16x3": 2.0 ** -15, "f16x3": 2.0 ** -21}


@pytest.mark.parametrize("precision", ["bf16x3", "f16x3"])
@pytest.mark.parametrize("preset", ["v1", "v2star"])
def test_split_packing(pkg, preset, precision):
    """Split-precision layers: the packed hi/lo planes reconstruct every weight to ~2^-16
    (bf16x3) / ~2^-22 (f16x3, after the layer's 2^-ew) relative, in the fragment order of
    conv_bf16x3.hip (tile 6 for the 256-row layer convs, tile 5 for the other M >= 128, tiles 1 / 2
    below)."""
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=31)
    h = host_handle(pkg, cfg, precision)
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    # tile -> (WAVES_M, WM, TPC)
    WAVES = {0: (2, 2, 4), 1: (1, 2, 2), 2: (1, 1, 4), 3: (2, 2, 2), 4: (2, 1, 4), 5: (2, 2, 2),
             6: (4, 2, 2)}
    n_checked = 0
    for mod in ["conv_pre", "mrfs.0.resblocks.2.convs1.1", "mrfs.1.resblocks.0.convs2.1",
                "mrfs.2.resblocks.1.convs1.0", "mrfs.3.resblocks.2.convs2.1"]:
        info, packed, bias = h.packed_layer(mod)
        W = sd[mod + ".weight"]
        cout, cin, k = W.shape
        if info["CK"] != 16:  # fp32 layer (C < 32 stage)
            assert cout < 32
            continue
        n_checked += 1
        wm_, WM, TPC = WAVES[info["tile"]]
        MT = info["MT"]
        n_g, n_tg = -(-cin // 16), -(-k // TPC)
        assert info["n_chunks"] == n_g * n_tg
        u = packed.view(np.uint16).reshape(info["m_tiles"], n_g, n_tg, TPC, 2, wm_, WM, 64, 8)
        hi = dec(u[:, :, :, :, 0], precision, info["ew"])
        lo = dec(u[:, :, :, :, 1], precision, info["ew"])
        if precision == "f16x3":  # the layer's max |w| lands in [2^14, 2^15) of f16
            assert 2.0 ** 14 <= np.abs(W).max() * 2.0 ** info["ew"] < 2.0 ** 15, mod
        rec = np.zeros((info["m_tiles"] * MT, n_g * 16, n_tg * TPC), np.float64)
        lane = np.arange(64)
        for mt in range(info["m_tiles"]):
            for g in range(n_g):
                for tg in range(n_tg):
                    for jj in range(TPC):
                        for wv in range(wm_):
                            for wm in range(WM):
                                rows = mt * MT + wv * 32 * WM + wm * 32 + (lane & 31)
                                for e in range(8):
                                    cis = g * 16 + 8 * (lane >> 5) + e
                                    val = (hi[mt, g, tg, jj, wv, wm, :, e].astype(np.float64)
                                           + lo[mt, g, tg, jj, wv, wm, :, e])
                                    rec[rows, cis, tg * TPC + jj] = val
        rec = rec[:cout, :cin, :k]
        err = np.abs(rec - W).max() / np.abs(W).max()
        assert err < SPLIT_TOL[precision], (mod, err)
        assert np.array_equal(bias[:cout], sd[mod + ".bias"])
    assert n_checked >= 2


def unpack_bf16x3(info, packed, waves, precision="bf16x3"):
    """Invert conv_bf16x3's fragment order → Wt[row][ci][tap] (hi + lo, float64)."""
    wm_, WM, TPC = waves
    MT = info["MT"]
    n_chunks, KT = info["n_chunks"], info["KT"]
    n_tg = -(-KT // TPC)
    n_g = n_chunks // n_tg
    u = packed.view(np.uint16).reshape(info["m_tiles"], n_g, n_tg, TPC, 2, wm_, WM, 64, 8)
    val = dec(u[:, :, :, :, 0], precision, info["ew"]) + dec(u[:, :, :, :, 1], precision, info["ew"])
    Wt = np.zeros((info["m_tiles"] * MT, n_g * 16, n_tg * TPC))
    lane = np.arange(64)
    for mt in range(info["m_tiles"]):
        for g in range(n_g):
            for tg in range(n_tg):
                for jj in range(TPC):
                    for wv in range(wm_):
                        for wm in range(WM):
                            rows = mt * MT + wv * 32 * WM + wm * 32 + (lane & 31)
                            for e in range(8):
                                Wt[rows, g * 16 + 8 * (lane >> 5) + e, tg * TPC + jj] = \
                                    val[mt, g, tg, jj, wv, wm, :, e]
    return Wt[: info["M"], :, :KT]


@pytest.mark.parametrize("precision", ["bf16x3", "f16x3"])
def test_split_polyphase_upsampler_packing(pkg, precision):
    cfg = C.NONEXACT  # odd k-u on the first stages
    sd = C.make_state_dict(cfg, seed=41)
    h = host_handle(pkg, cfg, precision)
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    waves = {0: (2, 2, 4), 1: (1, 2, 2), 2: (1, 1, 4), 3: (2, 2, 2), 4: (2, 1, 4)}
    rng = np.random.default_rng(1)
    c0 = cfg.upsample_initial_channel
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        info, packed, bias = h.packed_layer(f"ups.{i}")
        cin, cout = c0 >> i, c0 >> (i + 1)
        assert info["kind"] == 1 and info["CK"] == 16
        Wt = unpack_bf16x3(info, packed, waves[info["tile"]], precision)[:, :cin]
        x = rng.standard_normal((cin, 9)).astype(np.float32)
        ref = F.conv_transpose1d(torch.from_numpy(x)[None], torch.from_numpy(sd[f"ups.{i}.weight"]),
                                 torch.from_numpy(sd[f"ups.{i}.bias"]), u, (k - u) // 2)[0].numpy()
        Lout, p = ref.shape[-1], (k - u) // 2
        N = (Lout - 1 + p) // u + 1
        g = emulate_conv(Wt, bias, x, -(info["KT"] - 1), 1, N)
        y = np.full((cout, Lout), np.nan)
        for m in range(cout * u):
            co, r = divmod(m, u)
            t = np.arange(N) * u + r - p
            ok = (t >= 0) & (t < Lout)
            y[co, t[ok]] = g[m, ok]
        assert not np.isnan(y).any()
        assert np.abs(y - ref).max() < 1e-3 * np.abs(ref).max()


def _lrelu(v):
    return np.where(v > 0, v, 0.1 * v)


def _conv_same(x, w, b, d):
    """Conv1d with 'same' zero padding (k odd), float64: x [C, L], w [C, C, k]."""
    k = w.shape[2]
    pad = (k - 1) // 2 * d
    xp = np.pad(x, ((0, 0), (pad, pad)))
    L = x.shape[1]
    out = np.repeat(b[:, None], L, axis=1).astype(np.float64)
    for j in range(k):
        out += w[:, :, j] @ xp[:, j * d:j * d + L]
    return out


@pytest.mark.parametrize("precision", ["bf16x3", "f16x3"])
@pytest.mark.parametrize("preset", ["v1", "v2star"])
def test_resblock_stream_packing_and_windowing(pkg, preset, precision):
    """Whole-ResBlock launches (resblock_bf16x3.hip) of the narrow stages: the packed A
    stream decodes (hi + lo, permuted channel slots) to every conv's weights, and the
    kernel's windowing (NWIN-column windows, garbage edges, centre W = NWIN - 2*halo,
    zero outside [0, len)) reproduces the un-windowed ResBlock, emulated in float64."""
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=43)
    h = host_handle(pkg, cfg, precision)
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    n_fused = 0
    for i in range(len(cfg.upsample_rates)):
        for j in range(len(cfg.resblock_kernel_sizes)):
            info, packed, bias = h.packed_resblock(i, j)
            Cst = cfg.upsample_initial_channel >> (i + 1)
            if not info["fused"]:
                assert Cst not in (32, 64) or preset != "v1"
                continue
            n_fused += 1
            assert info["fused"] == 1
            Cc, KT, n_conv = info["C"], info["KT"], info["n_conv"]
            assert Cc == Cst and KT == cfg.resblock_kernel_sizes[j]
            dils = cfg.resblock_dilation_sizes[j]
            assert n_conv == 2 * len(dils)
            # the first conv is exact on the whole window (margins staged from x): the halo
            # is the radius of the convs after it
            assert info["halo"] == sum((KT - 1) // 2 * d + (KT - 1) // 2 for d in dils) \
                - (KT - 1) // 2 * dils[0]
            # W is rounded down to a multiple of 4 (16-B aligned block origins)
            nwin = next(n for n in (256, 512, 1024) if 0 <= n - info["W"] - 2 * info["halo"] < 4)
            assert info["W"] % 4 == 0
            if Cc == 64:  # narrow 256-column window (2 blocks per CU) only for k = 3
                assert nwin == (256 if KT == 3 else 512)
            lane = np.arange(64)
            # resblock: [wave_m][conv][g][tap][plane][lane][8]
            u = packed.view(np.uint16).reshape(Cc // 32, n_conv, Cc // 16, KT, 2, 64, 8)
            Ws = []
            for e in range(n_conv):
                m, second = divmod(e, 2)
                mod = f"mrfs.{i}.resblocks.{j}.convs{2 if second else 1}.{m}"
                ew = h.packed_layer(mod)[0]["ew"]
                val = dec(u[:, :, :, :, 0], precision, ew) + dec(u[:, :, :, :, 1], precision, ew)
                W = sd[mod + ".weight"].astype(np.float64)
                rec = np.zeros_like(W)
                for wm in range(Cc // 32):
                    rows = wm * 32 + (lane & 31)
                    for g in range(Cc // 16):
                        for el in range(8):
                            ci = g * 16 + 4 * (lane >> 5) + (el & 3) + 8 * (el >> 2)
                            rec[rows, ci, :] = val[wm, e, g, :, lane, el]
                assert np.abs(rec - W).max() <= SPLIT_TOL[precision] * np.abs(W).max(), mod
                assert np.array_equal(bias[e * Cc:(e + 1) * Cc], sd[mod + ".bias"])
                Ws.append((rec, sd[mod + ".bias"].astype(np.float64)))
            # windowed emulation vs direct, on one short utterance (len < L)
            if j != len(cfg.resblock_kernel_sizes) - 1:
                continue
            rng = np.random.default_rng(5)
            L, ln = 3 * info["W"] // 2 + 37, 3 * info["W"] // 2 + 5
            x = rng.standard_normal((Cc, L))
            x[:, ln:] = 0.0

            def resblock(xx, valid):
                for m in range(len(dils)):
                    (w1, b1), (w2, b2) = Ws[2 * m], Ws[2 * m + 1]
                    t = _lrelu(_conv_same(_lrelu(xx) * valid, w1, b1, dils[m])) * valid
                    xx = xx + _conv_same(t, w2, b2, 1)
                return xx

            def resblock_window(xe, ve, r0):
                """the kernel's window: the first conv reads r0 columns of x past either
                edge (the LDS margins) and is kept on the window only; later convs see the
                window alone (zero padding of the window itself emulates the arbitrary data
                past its edges: any value gives the same centre)"""
                (w1, b1), (w2, b2) = Ws[0], Ws[1]
                t = _conv_same(_lrelu(xe) * ve, w1, b1, dils[0])[:, r0:r0 + nwin]
                xx, valid = xe[:, r0:r0 + nwin], ve[r0:r0 + nwin]
                xx = xx + _conv_same(_lrelu(t) * valid, w2, b2, 1)
                for m in range(1, len(dils)):
                    (w1, b1), (w2, b2) = Ws[2 * m], Ws[2 * m + 1]
                    t = _lrelu(_conv_same(_lrelu(xx) * valid, w1, b1, dils[m])) * valid
                    xx = xx + _conv_same(t, w2, b2, 1)
                return xx

            direct = resblock(x[:, :ln], np.ones(ln))
            out = np.zeros((Cc, ln))
            r0 = (KT - 1) // 2 * dils[0]
            for t0 in range(0, ln, info["W"]):
                ws = t0 - info["halo"]
                cols = ws - r0 + np.arange(nwin + 2 * r0)
                valid = ((cols >= 0) & (cols < ln)).astype(np.float64)
                xw = np.where(valid > 0, x[:, np.clip(cols, 0, L - 1)], 0.0)
                yw = resblock_window(xw, valid, r0)
                c0, c1 = info["halo"], info["halo"] + min(info["W"], ln - t0)
                out[:, t0:t0 + (c1 - c0)] = yw[:, c0:c1]
            assert np.abs(out - direct).max() < 1e-9
    assert n_fused >= (7 if preset == "v1" else 1)


def _bf16_rne(a):
    """float32 → bf16 round-to-nearest-even, returned as float32 (numpy)."""
    u = np.asarray(a, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32) << 16
    return r.view(np.float32)


@pytest.mark.parametrize("preset", ["v1", "v2star"])
def test_bf16w_packing(pkg, preset):
    """HFG_DTYPE_BF16W: every conv weight is rounded to bf16 (nearest-even) when committed —
    the split layers (f16 halves of w 2^ew) have all-zero lo planes and hi planes exactly
    bf16(W) 2^ew (8 significant bits fit f16's 11); the fp32 layers (conv_post, C < 32
    stages) hold the same bf16-valued weights; biases stay fp32."""
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=41)
    h = host_handle(pkg, cfg, "bf16w")
    for k, v in sd.items():
        h.set_weight(k, torch.from_numpy(v))
    h.commit()
    h.commit()  # idempotent
    n_split = n_fp32 = 0
    for mod in ["conv_pre", "ups.0", "mrfs.0.resblocks.2.convs1.1", "mrfs.1.resblocks.0.convs2.1",
                "mrfs.3.resblocks.2.convs2.1", "conv_post"]:
        info, packed, bias = h.packed_layer(mod)
        W = sd[mod + ".weight"]
        if mod.startswith("ups."):  # bias repeated per polyphase row
            assert set(np.unique(bias)) - {0.0} <= set(sd[mod + ".bias"]), mod
        else:
            assert np.array_equal(bias[:W.shape[0]], sd[mod + ".bias"]), mod
        if info["CK"] == 16:
            assert info["tile"] != 0, mod
            n_split += 1
            u = packed.view(np.uint16)
            TPC = {0: 4, 1: 2, 2: 4, 3: 2, 4: 4, 5: 2, 6: 2}[info["tile"]]
            planes = u.reshape(-1, TPC, 2, u.size // (info["m_tiles"] * info["n_chunks"] * TPC * 2))
            assert not planes[:, :, 1].any(), f"{mod}: lo plane not zero"
            hi = np.sort(dec(planes[:, :, 0], "bf16w", info["ew"]).astype(np.float32).ravel())
            ref = np.sort(np.concatenate([_bf16_rne(W).ravel(),
                                          np.zeros(hi.size - W.size, np.float32)]))
            assert np.array_equal(hi, ref), mod
        else:
            n_fp32 += 1
            vals = np.asarray(packed, np.float32)
            assert not (vals.view(np.uint32) & 0xFFFF).any(), f"{mod}: weight not bf16-valued"
            nz = np.sort(vals[vals != 0])
            ref = _bf16_rne(W).ravel()
            assert np.array_equal(nz, np.sort(ref[ref != 0])), mod
    assert n_split >= 3 and n_fp32 >= 1


def test_layer_exponent_entry_commits_or_reports(pkg):
    """hfg_debug_layer_exponent: with a weight missing it returns the commit's
    error instead of a stale 0; info-only hfg_debug_packed_layer fills exactly 10 entries and
    does not commit."""
    import ctypes
    cfg = C.V2STAR
    h = host_handle(pkg, cfg, precision="f16x3")
    lib = pkg.load_library()
    sd = C.make_state_dict(cfg, seed=6)
    keys = list(sd)
    for k in keys[:-1]:
        h.set_weight(k, torch.from_numpy(sd[k]))
    ew = ctypes.c_int(-99)
    assert lib.hfg_debug_layer_exponent(h.ptr, b"ups.1", ctypes.byref(ew)) != 0
    assert ew.value == -99
    info = (ctypes.c_int64 * 11)(*([-7] * 11))
    assert lib.hfg_debug_packed_layer(h.ptr, b"ups.1", None, 0, info) == 0
    assert info[10] == -7 and info[9] > 0
    h.set_weight(keys[-1], torch.from_numpy(sd[keys[-1]]))
    assert lib.hfg_debug_layer_exponent(h.ptr, b"ups.1", ctypes.byref(ew)) == 0
    w = sd["ups.1.weight"]
    assert ew.value == 15 - int(np.frexp(np.abs(w).max())[1])


def test_removed_knob_value_is_refused(pkg):
    """UPS_FRAMES=0 (the polyphase-only schedule, removed in round 4) is refused by the
    schedule-override entry point instead of silently running the default schedule
    (ADVICE r04); unknown knobs and out-of-range values are refused too."""
    lib = pkg.load_library()
    c = pkg.make_config(80, [8, 8, 2, 2], [16, 16, 4, 4], 512, [3, 7, 11], [[1, 3, 5]] * 3)
    try:
        assert lib.hfg_debug_schedule_set(b"UPS_FRAMES", 0) == -22
        assert b"UPS_FRAMES" in lib.hfg_last_error() and b"removed" in lib.hfg_last_error()
        assert lib.hfg_debug_schedule_set(b"NO_SUCH_KNOB", 1) == -22
        assert lib.hfg_debug_schedule_set(b"SMALL_TILE", 2) == -22
        assert pkg.schedule_overrides() == {}
        assert lib.hfg_debug_schedule_set(b"UPS_FRAMES", 2) == 0
        assert pkg.schedule_overrides() == {"UPS_FRAMES": 2}
        h = ctypes.c_void_p()
        assert lib.hfg_create(ctypes.byref(c), -1, ctypes.byref(h)) == 0
        lib.hfg_destroy(h)
    finally:
        pkg.schedule_clear()
    assert pkg.schedule_overrides() == {}


def _fused_flag(pkg, precision="f16x3"):
    """info[0] of hfg_debug_packed_resblock for stage 3, ResBlock 0: 1 when the stage runs
    whole-ResBlock launches, 0 layer by layer (the FUSED_RB schedule choice)."""
    cfg = C.V1
    h = host_handle(pkg, cfg, precision)
    for k, v in C.make_state_dict(cfg, seed=3).items():
        h.set_weight(k, torch.from_numpy(v))
    info = (ctypes.c_int64 * 8)()
    assert h.lib.hfg_debug_packed_resblock(h.ptr, 3, 0, None, 0, info) == 0
    return int(info[0])


def test_schedule_ignores_environment(pkg, monkeypatch, sched):
    """The production handle's schedule does not depend on the caller's environment
    (VERDICT r05 item 8): HFG_FUSED_RB=0 in the environment leaves the whole-ResBlock
    schedule on; the override entry point (the tests' and A/B runs' path) switches it."""
    assert _fused_flag(pkg) == 1
    monkeypatch.setenv("HFG_FUSED_RB", "0")
    assert _fused_flag(pkg) == 1
    sched("FUSED_RB", 0)
    assert _fused_flag(pkg) == 0
    pkg.schedule_clear("FUSED_RB")
    assert _fused_flag(pkg) == 1
