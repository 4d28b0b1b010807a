"""Rectification: initUndistortRectifyMap CV_16SC2 + remap INTER_LINEAR.

OpenCV 3.0 is absent and the reference has no fixtures for P/Main.cpp:351-359,
so parity against OpenCV is UNPINNED.  The oracle restatement
(oracle/rectify_oracle.c) is pinned here by known answers -- an identity
calibration reproduces the source, an integer principal-point shift gives a
shifted copy with zeros entering, a half-pixel shift gives the rounded mean of
neighbours -- and by an independent numpy restatement of the fixed-point
bilinear remap; the GPU kernels must equal the oracle bit for bit.
"""
import numpy as np
import pytest

from oracle_lib import load_oracle, oracle_rectify_map, oracle_rectify_params, oracle_remap
from unsynchronized_stereo_vision_proj325_amd import _lib
from unsynchronized_stereo_vision_proj325_amd.rectify import rectify_params, synthetic_calibration


def numpy_remap(src, m1, m2):
    """Independent restatement of remap INTER_LINEAR / BORDER_CONSTANT 0 (fixed point, 5+15 bits)."""
    src = src if src.ndim == 3 else src[:, :, None]
    sH, sW, cn = src.shape
    sx = m1[..., 0].astype(np.int64)
    sy = m1[..., 1].astype(np.int64)
    ty = (m2 >> 5).astype(np.int64)
    tx = (m2 & 31).astype(np.int64)
    w = [(32 - ty) * (32 - tx) * 32, (32 - ty) * tx * 32, ty * (32 - tx) * 32, ty * tx * 32]
    acc = np.zeros(sx.shape + (cn,), dtype=np.int64)
    for k, (dy, dx) in enumerate([(0, 0), (0, 1), (1, 0), (1, 1)]):
        yy, xx = sy + dy, sx + dx
        ok = (yy >= 0) & (yy < sH) & (xx >= 0) & (xx < sW)
        v = src[np.clip(yy, 0, sH - 1), np.clip(xx, 0, sW - 1)].astype(np.int64)
        acc += np.where(ok[..., None], v, 0) * w[k][..., None]
    out = np.clip((acc + (1 << 14)) >> 15, 0, 255)
    outside = (sx >= sW) | (sx + 1 < 0) | (sy >= sH) | (sy + 1 < 0)
    out[outside] = 0
    out = out.astype(np.uint8)
    return out[..., 0] if cn == 1 else out


def pinhole(f, cx, cy):
    return np.array([[f, 0, cx], [0, f, cy], [0, 0, 1.0]])


def test_identity_calibration_reproduces_source():
    K = pinhole(500.0, 320.0, 240.0)
    m1, m2 = oracle_rectify_map(oracle_rectify_params(K, None, None, K), 64, 48)
    ys, xs = np.mgrid[0:48, 0:64]
    assert np.array_equal(m1[..., 0], xs) and np.array_equal(m1[..., 1], ys) and not m2.any()
    src = np.random.default_rng(0).integers(0, 256, (48, 64, 3), dtype=np.uint8)
    assert np.array_equal(oracle_remap(src, m1, m2), src)


@pytest.mark.parametrize("shift", [3, -5])
def test_integer_principal_point_shift(shift):
    K = pinhole(500.0, 320.0, 240.0)
    P = np.hstack([pinhole(500.0, 320.0 + shift, 240.0), np.zeros((3, 1))])
    m1, m2 = oracle_rectify_map(oracle_rectify_params(K, None, None, P), 40, 20)
    src = np.random.default_rng(1).integers(1, 256, (20, 40), dtype=np.uint8)
    out = oracle_remap(src, m1, m2)
    exp = np.zeros_like(src)
    if shift > 0:
        exp[:, shift:] = src[:, :-shift]
    else:
        exp[:, :shift] = src[:, -shift:]
    assert np.array_equal(out, exp)


def test_half_pixel_shift_rounds_the_mean():
    K = pinhole(400.0, 100.0, 50.0)
    P = pinhole(400.0, 100.5, 50.0)
    m1, m2 = oracle_rectify_map(oracle_rectify_params(K, None, None, P), 30, 10)
    assert ((m2 & 31) == 16).all() and ((m2 >> 5) == 0).all()
    src = np.random.default_rng(2).integers(0, 256, (10, 30), dtype=np.uint8)
    out = oracle_remap(src, m1, m2).astype(int)
    s = src.astype(int)
    assert np.array_equal(out[:, 1:], (s[:, :-1] + s[:, 1:] + 1) >> 1)
    assert np.array_equal(out[:, 0], (s[:, 0] + 1) >> 1)  # left tap outside the image reads 0


@pytest.mark.parametrize("cn", [1, 3])
def test_oracle_remap_matches_numpy_restatement(cn):
    rng = np.random.default_rng(3 + cn)
    sH, sW, H, W = 37, 53, 29, 41
    src = rng.integers(0, 256, (sH, sW) if cn == 1 else (sH, sW, cn), dtype=np.uint8)
    m1 = np.stack([rng.integers(-4, sW + 3, (H, W)), rng.integers(-4, sH + 3, (H, W))], -1).astype(np.int16)
    m2 = rng.integers(0, 1024, (H, W)).astype(np.uint16)
    assert np.array_equal(oracle_remap(src, m1, m2), numpy_remap(src, m1, m2))


def test_invert3_against_numpy():
    lib = load_oracle()
    rng = np.random.default_rng(5)
    for _ in range(50):
        m = rng.normal(size=(3, 3))
        out = np.zeros(9)
        assert lib.usv_oracle_invert3(m.ctypes.data, out.ctypes.data) == 1
        np.testing.assert_allclose(out.reshape(3, 3), np.linalg.inv(m), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("ndist", [0, 4, 5, 8, 12])
def test_library_params_equal_oracle(ndist):
    """usv_rectify_params (host code of libusv.so; no GPU needed) == the oracle, bit for bit."""
    rng = np.random.default_rng(10 + ndist)
    (K, dist, R, P), _ = synthetic_calibration(640, 480, seed=ndist)
    d = rng.uniform(-0.2, 0.2, ndist)
    got = rectify_params(K, d, R, P)
    ref = oracle_rectify_params(K, d, R, P)
    assert np.array_equal(got, ref)


def test_library_rejects_bad_calibration():
    lib = _lib.load()
    out = np.zeros(25)
    K = pinhole(1.0, 0.0, 0.0)
    sing = np.zeros((3, 4))
    assert lib.usv_rectify_params(K.ctypes.data, None, 0, None, sing.ctypes.data, 4, out.ctypes.data) == \
        _lib.USV_ERR_INVALID_ARG
    d = np.zeros(6)
    assert lib.usv_rectify_params(K.ctypes.data, d.ctypes.data, 6, None, K.ctypes.data, 3, out.ctypes.data) == \
        _lib.USV_ERR_INVALID_ARG


# ---------------------------------------------------------------- GPU parity
def _dev_maps(gpu, K, dist, R, P, W, H):
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier
    return Rectifier(K, dist, R, P, (W, H), device=gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,seed,ndist", [(640, 480, 0, 5), (1920, 1080, 1, 5), (333, 97, 2, 8),
                                            (1000, 700, 3, 12), (64, 64, 4, 0)])
def test_gpu_map_bitexact(gpu, W, H, seed, ndist):
    (K, dist, R, P), _ = synthetic_calibration(W, H, seed=seed)
    d = np.resize(dist, ndist) if ndist else None
    rect = _dev_maps(gpu, K, d, R, P, W, H)
    m1, m2 = rect.maps_numpy()
    r1, r2 = oracle_rectify_map(oracle_rectify_params(K, d, R, P), W, H)
    assert np.array_equal(m1, r1), int((m1 != r1).sum())
    assert np.array_equal(m2, r2), int((m2 != r2).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
@pytest.mark.parametrize("W,H", [(640, 480), (1920, 1080), (97, 41), (3, 2)])
def test_gpu_remap_bitexact(gpu, cn, W, H):
    import torch
    (K, dist, R, P), _ = synthetic_calibration(W, H, seed=W + cn)
    rect = _dev_maps(gpu, K, dist, R, P, W, H)
    rng = np.random.default_rng(W * H + cn)
    src = rng.integers(0, 256, (H, W) if cn == 1 else (H, W, cn), dtype=np.uint8)
    got = rect(torch.from_numpy(src).to(gpu)).cpu().numpy()
    m1, m2 = rect.maps_numpy()
    assert np.array_equal(got, oracle_remap(src, m1, m2))


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
def test_gpu_remap_wild_maps_and_pitched_output(gpu, cn):
    """Maps pointing far outside the source (negative, past the border), odd widths, pitched dst."""
    import ctypes
    import torch
    rng = np.random.default_rng(77 + cn)
    sH, sW, H, W = 50, 70, 33, 45
    src = rng.integers(0, 256, (sH, sW) if cn == 1 else (sH, sW, cn), dtype=np.uint8)
    m1 = np.stack([rng.integers(-300, 400, (H, W)), rng.integers(-300, 400, (H, W))], -1).astype(np.int16)
    m1[::3] = np.stack([rng.integers(-2, sW + 1, (H, W)), rng.integers(-2, sH + 1, (H, W))], -1)[::3]
    m2 = rng.integers(0, 1024, (H, W)).astype(np.uint16)
    d_src = torch.from_numpy(src).to(gpu)
    d_m1 = torch.from_numpy(m1).to(gpu)
    d_m2 = torch.from_numpy(m2.view(np.int16)).to(gpu)
    big = torch.zeros((H, (W + 13) * cn), dtype=torch.uint8, device=gpu)
    lib = _lib.load()
    st = lib.usv_remap_linear_u8(d_src.data_ptr(), sW, sH, sW * cn, cn, d_m1.data_ptr(), d_m2.data_ptr(), W, H,
                                 big.data_ptr(), big.stride(0), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == _lib.USV_OK
    got = big[:, :W * cn].cpu().numpy()
    ref = oracle_remap(src, m1, m2).reshape(H, W * cn)
    assert np.array_equal(got, ref)
    assert not big[:, W * cn:].any()  # nothing written past the row


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
def test_gpu_rectify_pair_equals_two_remaps(gpu, cn):
    import torch
    from unsynchronized_stereo_vision_proj325_amd.rectify import rectify_pair
    W, H = 640, 480
    (cl, cr) = synthetic_calibration(W, H, seed=9)
    rl, rr = _dev_maps(gpu, *cl, W, H), _dev_maps(gpu, *cr, W, H)
    rng = np.random.default_rng(cn)
    shape = (H, W) if cn == 1 else (H, W, cn)
    sl = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    sr = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    ol, orr = rectify_pair(rl, rr, sl, sr)
    assert torch.equal(ol, rl(sl)) and torch.equal(orr, rr(sr))


# ---------------------------------------------------------------- packed map (usv_remap_pack_map)
PACK_MAX = 2046


def numpy_pack_map(m1, m2, sW, sH):
    """include/usv.h usv_remap_pack_map restated: fraction | (sx + 1) << 10 | (sy + 1) << 21, a pixel with
    no tap inside the source stored as 2047 / 2047."""
    sx = m1[..., 0].astype(np.int64)
    sy = m1[..., 1].astype(np.int64)
    any_ = (sx < sW) & (sx + 1 >= 0) & (sy < sH) & (sy + 1 >= 0)
    ex = np.where(any_, sx + 1, 2047)
    ey = np.where(any_, sy + 1, 2047)
    return ((m2.astype(np.int64) & 1023) | (ex << 10) | (ey << 21)).astype(np.uint32)


def numpy_unpack_map(pm):
    pm = pm.astype(np.int64)
    m1 = np.stack([((pm >> 10) & 2047) - 1, (pm >> 21) - 1], -1).astype(np.int16)
    return m1, (pm & 1023).astype(np.uint16)


def _wild_maps(rng, sW, sH, W, H):
    m1 = np.stack([rng.integers(-3000, 4000, (H, W)), rng.integers(-3000, 4000, (H, W))], -1).astype(np.int16)
    m1[::3] = np.stack([rng.integers(-2, sW + 1, (H, W)), rng.integers(-2, sH + 1, (H, W))], -1)[::3]
    m1[1::3, ::2] = np.stack([rng.integers(-1, sW, (H, W)), rng.integers(-1, sH, (H, W))], -1)[1::3, ::2]
    m2 = rng.integers(0, 1024, (H, W)).astype(np.uint16)
    return m1, m2


@pytest.mark.parametrize("cn", [1, 3])
@pytest.mark.parametrize("sW,sH", [(70, 50), (PACK_MAX, 3), (5, PACK_MAX)])
def test_packed_map_format_preserves_remap(cn, sW, sH):
    """The packed format loses nothing remap can see: the oracle's remap through the decoded map equals
    its remap through the original one, for maps far outside the source, on the border and inside."""
    rng = np.random.default_rng(sW + 7 * sH + cn)
    H, W = 9, 31
    src = rng.integers(0, 256, (sH, sW) if cn == 1 else (sH, sW, cn), dtype=np.uint8)
    m1, m2 = _wild_maps(rng, sW, sH, W, H)
    d1, d2 = numpy_unpack_map(numpy_pack_map(m1, m2, sW, sH))
    assert np.array_equal(oracle_remap(src, d1, d2), oracle_remap(src, m1, m2))


def test_packed_map_rejects_large_sources():
    lib = _lib.load()
    # argument checks run before any device work: no GPU needed
    assert lib.usv_remap_pack_map(8, 8, 4, 4, PACK_MAX + 1, 10, 8, None) == _lib.USV_ERR_UNSUPPORTED
    assert lib.usv_remap_pack_map(8, 8, 4, 4, 10, PACK_MAX + 1, 8, None) == _lib.USV_ERR_UNSUPPORTED
    assert lib.usv_remap_pack_map(None, 8, 4, 4, 10, 10, 8, None) == _lib.USV_ERR_INVALID_ARG
    assert lib.usv_remap_packed_u8(8, PACK_MAX + 1, 4, PACK_MAX + 1, 1, 8, 4, 4, 8, 4, None) == \
        _lib.USV_ERR_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
def test_gpu_packed_map_and_remap_wild(gpu, cn):
    """usv_remap_pack_map equals the numpy restatement; remapping through it (pitched output, odd
    width) equals the oracle's remap through the original map pair."""
    import ctypes
    import torch
    rng = np.random.default_rng(99 + cn)
    sH, sW, H, W = 50, 70, 33, 45
    src = rng.integers(0, 256, (sH, sW) if cn == 1 else (sH, sW, cn), dtype=np.uint8)
    m1, m2 = _wild_maps(rng, sW, sH, W, H)
    d_src = torch.from_numpy(src).to(gpu)
    d_m1 = torch.from_numpy(m1).to(gpu)
    d_m2 = torch.from_numpy(m2.view(np.int16)).to(gpu)
    pm = torch.zeros((H, W), dtype=torch.int32, device=gpu)
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.usv_remap_pack_map(d_m1.data_ptr(), d_m2.data_ptr(), W, H, sW, sH, pm.data_ptr(), s) == _lib.USV_OK
    assert np.array_equal(pm.cpu().numpy().view(np.uint32), numpy_pack_map(m1, m2, sW, sH))
    big = torch.zeros((H, (W + 13) * cn), dtype=torch.uint8, device=gpu)
    assert lib.usv_remap_packed_u8(d_src.data_ptr(), sW, sH, sW * cn, cn, pm.data_ptr(), W, H, big.data_ptr(),
                                   big.stride(0), s) == _lib.USV_OK
    got = big[:, :W * cn].cpu().numpy()
    assert np.array_equal(got, oracle_remap(src, m1, m2).reshape(H, W * cn))
    assert not big[:, W * cn:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
@pytest.mark.parametrize("W,H", [(1920, 1080), (97, 41)])
def test_gpu_rectifier_packed_equals_unpacked(gpu, cn, W, H):
    import torch
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair
    cl, cr = synthetic_calibration(W, H, seed=5 + cn)
    pk = [Rectifier(*c, (W, H), device=gpu) for c in (cl, cr)]
    up = [Rectifier(*c, (W, H), device=gpu, packed=False) for c in (cl, cr)]
    assert pk[0].pmap is not None and up[0].pmap is None
    rng = np.random.default_rng(W + cn)
    shape = (H, W) if cn == 1 else (H, W, cn)
    sl = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    sr = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    assert torch.equal(pk[0](sl), up[0](sl))
    a, b = rectify_pair(pk[0], pk[1], sl, sr)
    c, d = rectify_pair(up[0], up[1], sl, sr)
    assert torch.equal(a, c) and torch.equal(b, d)
    m1, m2 = up[1].maps_numpy()
    assert np.array_equal(b.cpu().numpy(), oracle_remap(sr.cpu().numpy(), m1, m2))


@pytest.mark.gpu
def test_gpu_rectifier_large_source_uses_map_pair(gpu):
    """A source wider than 2046 columns has no packed form: the Rectifier keeps the map pair."""
    import torch
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier
    W, H = 2100, 24
    (K, dist, R, P), _ = synthetic_calibration(W, H, seed=3)
    rect = Rectifier(K, dist, R, P, (W, H), device=gpu)
    assert rect.pmap is None
    src = np.random.default_rng(1).integers(0, 256, (H, W, 3), dtype=np.uint8)
    m1, m2 = rect.maps_numpy()
    assert np.array_equal(rect(torch.from_numpy(src).to(gpu)).cpu().numpy(), oracle_remap(src, m1, m2))


def _numpy_tile_boxes(pm, W, H, sW, sH, cn, tw=64, th=16, max_dw=3072):
    """usv_remap_tile_boxes restated: per 64 x 16 tile, the in-image box of every pixel's taps."""
    pm = pm.astype(np.uint32)
    sx = ((pm >> 10) & 2047).astype(np.int64) - 1
    sy = (pm >> 21).astype(np.int64) - 1
    any_tap = (sx < sW) & (sx + 1 >= 0) & (sy < sH) & (sy + 1 >= 0)
    out = []
    for ty in range(0, H, th):
        for tx in range(0, W, tw):
            m = any_tap[ty:ty + th, tx:tx + tw]
            if not m.any():
                out.append((0, 0))
                continue
            x, y = sx[ty:ty + th, tx:tx + tw][m], sy[ty:ty + th, tx:tx + tw][m]
            bx0, bx1 = max(int(x.min()), 0), min(int(x.max()) + 1, sW - 1)
            by0, by1 = max(int(y.min()), 0), min(int(y.max()) + 1, sH - 1)
            if not (bx1 > bx0 and by1 > by0):
                out.append((0, 0))
                continue
            rowdw = (((bx1 + 1) * cn + 3) >> 2) - ((bx0 * cn) >> 2) + 2
            h = by1 - by0 + 1
            out.append((bx0 | (by0 << 16), rowdw | (h << 16)) if rowdw <= 256 and rowdw * h <= max_dw else (0, 0))
    return np.array(out, dtype=np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
def test_gpu_tiled_remap_wild_maps(gpu, cn):
    """The LDS-tiled packed remap (usv_remap_tile_boxes + usv_remap_packed_tiled_u8) on wild maps -- tiles
    whose boxes are too large for LDS, taps outside the source, an odd width, pitched output -- equals the
    oracle's remap; the boxes equal the numpy restatement."""
    import ctypes
    import torch
    rng = np.random.default_rng(199 + cn)
    sH, sW, H, W = 150, 170, 45, 133
    src = rng.integers(0, 256, (sH, sW) if cn == 1 else (sH, sW, cn), dtype=np.uint8)
    m1, m2 = _wild_maps(rng, sW, sH, W, H)
    # the top-left quarter as a smooth, small-box warp so the LDS path runs too
    yy, xx = np.mgrid[0:H // 2, 0:W // 2]
    m1[:H // 2, :W // 2, 0] = (xx * 1.1 + 3).astype(np.int16)
    m1[:H // 2, :W // 2, 1] = (yy * 0.9 + 2 + xx // 40).astype(np.int16)
    d_src = torch.from_numpy(src).to(gpu)
    d_m1 = torch.from_numpy(m1).to(gpu)
    d_m2 = torch.from_numpy(m2.view(np.int16)).to(gpu)
    pm = torch.zeros((H, W), dtype=torch.int32, device=gpu)
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.usv_remap_pack_map(d_m1.data_ptr(), d_m2.data_ptr(), W, H, sW, sH, pm.data_ptr(), s) == _lib.USV_OK
    tiles = ((W + 63) // 64) * ((H + 15) // 16)
    boxes = torch.zeros((tiles, 2), dtype=torch.int32, device=gpu)
    assert lib.usv_remap_tile_boxes(pm.data_ptr(), W, H, sW, sH, cn, boxes.data_ptr(), s) == _lib.USV_OK
    want = _numpy_tile_boxes(pm.cpu().numpy().view(np.uint32), W, H, sW, sH, cn)
    assert np.array_equal(boxes.cpu().numpy().view(np.uint32), want)
    assert (want[:, 1] != 0).any() and (want[:, 1] == 0).any()  # both paths exercised
    big = torch.zeros((H, (W + 13) * cn), dtype=torch.uint8, device=gpu)
    assert lib.usv_remap_packed_tiled_u8(d_src.data_ptr(), sW, sH, sW * cn, cn, pm.data_ptr(), boxes.data_ptr(), W,
                                         H, big.data_ptr(), big.stride(0), s) == _lib.USV_OK
    got = big[:, :W * cn].cpu().numpy()
    assert np.array_equal(got, oracle_remap(src, m1, m2).reshape(H, W * cn))
    assert not big[:, W * cn:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [1, 3])
def test_gpu_rectifier_tiled_equals_direct(gpu, cn):
    """1080p synthetic calibration: the tiled packed remap (opt-in, tiled=True) equals the direct packed
    remap and the oracle, single camera and pair."""
    import torch
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair
    W, H = 1920, 1080
    cl, cr = synthetic_calibration(W, H, seed=17 + cn)
    tl = [Rectifier(*c, (W, H), device=gpu, tiled=True) for c in (cl, cr)]
    dl = [Rectifier(*c, (W, H), device=gpu) for c in (cl, cr)]
    rng = np.random.default_rng(3 * cn)
    shape = (H, W) if cn == 1 else (H, W, cn)
    sl = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    sr = torch.from_numpy(rng.integers(0, 256, shape, dtype=np.uint8)).to(gpu)
    assert torch.equal(tl[0](sl), dl[0](sl))
    a, b = rectify_pair(tl[0], tl[1], sl, sr)
    c, d = rectify_pair(dl[0], dl[1], sl, sr)
    assert torch.equal(a, c) and torch.equal(b, d)
    assert (tl[0].boxes(cn).cpu().numpy()[:, 1] != 0).mean() > 0.9  # nearly every tile on the LDS path
    m1, m2 = dl[1].maps_numpy()
    assert np.array_equal(b.cpu().numpy(), oracle_remap(sr.cpu().numpy(), m1, m2))


def test_tiled_remap_argument_checks():
    lib = _lib.load()  # argument checks run before any device work: no GPU needed
    assert lib.usv_remap_tile_boxes(None, 8, 8, 8, 8, 3, 8, None) == _lib.USV_ERR_INVALID_ARG
    assert lib.usv_remap_tile_boxes(8, 8, 8, 8, 8, 2, 8, None) == _lib.USV_ERR_UNSUPPORTED
    assert lib.usv_remap_tile_boxes(8, 8, 8, PACK_MAX + 1, 8, 3, 8, None) == _lib.USV_ERR_UNSUPPORTED
    assert lib.usv_remap_packed_tiled_u8(8, 8, 8, 24, 3, 8, None, 8, 8, 8, 24, None) == _lib.USV_ERR_INVALID_ARG
    assert lib.usv_rectify_pair_packed_tiled_u8(8, 8, 8, 8, 24, 3, 8, 8, 8, None, 8, 8, 8, 8, 24, None) == \
        _lib.USV_ERR_INVALID_ARG
