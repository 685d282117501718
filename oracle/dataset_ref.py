"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's image
preprocessing, the checker for the HIP data pipeline.

Reference: ``CellSegmentationDataset.__getitem__`` / ``normalize_microscopy_image``
(/root/reference/dataset.py:30-66):

    image = cv2.resize(image, img_size, interpolation=cv2.INTER_AREA)        # :51
    mask  = cv2.resize(mask,  img_size, interpolation=cv2.INTER_NEAREST)     # :52
    p_low, p_high = np.percentile(image, [2, 98])                           # :33
    image_clipped = np.clip(image, p_low, p_high)                           # :34
    image_clahe = cv2.createCLAHE(2.0, (8, 8)).apply(image_clipped.astype(np.uint8))  # :37-38
    image_norm = (image_clahe - image_clahe.min()) / (image_clahe.max() - image_clahe.min() + 1e-8)  # :41
    mask = (mask > 0).astype(np.float32)                                    # :61

and the two deterministic transforms of ``CellAugmenter`` (dataset.py:147-152):
``A.RandomRotate90`` (np.rot90 by k) and ``A.VerticalFlip``.

Third-party algorithms restated (neither OpenCV nor albumentations is
installed here, and the reference ships no image fixtures, so the cv2 parts
are PARITY UNPINNED; numpy's percentile is pinned against numpy itself):

* ``np.percentile`` (numpy 2.2, method='linear'): virtual index
  h = (n-1) q/100, v[floor] + (v[ceil]-v[floor]) * frac, numpy's _lerp form
  (``b - (b-a)(1-t)`` for t >= 0.5), float64.
* ``cv2.resize`` INTER_AREA, downscaling (OpenCV 4.x imgproc/src/resize.cpp):
  integer factors: ``resizeAreaFast_`` = integer block sum * (1/area) in float,
  ``cvRound``; otherwise ``computeResizeAreaTab`` coverage weights (float
  alpha per source column / row) accumulated horizontally then vertically in
  float, ``cvRound``.  Enlarging (either axis): resizeGeneric_ with the
  area_mode linear coefficients, fixed point (``resize_area_up_u8``).
  INTER_NEAREST: ``sx = min(floor(dx * (ssize/dsize)), ssize-1)``.
* ``cv2.CLAHE`` (imgproc/src/clahe.cpp, 8-bit path): tile grid 8x8 (BORDER_REFLECT_101
  padding when either side is not a multiple of the grid: both sides by
  ``grid - size % grid``, so a side that is a multiple gains a whole tile), clip limit max(int(2.0 * tileArea / 256), 1),
  excess redistributed as ``clipped // 256`` per bin + a residual every
  ``max(256 // residual, 1)`` bins, LUT = saturate(round(cumsum * 255 / tileArea)),
  bilinear interpolation between the 4 nearest tile LUTs in float
  (``txf = x / tileW - 0.5``), ``cvRound``.
"""
from __future__ import annotations

import math

import numpy as np


def percentile_linear(img: np.ndarray, q: float) -> float:
    """np.percentile(img, q) (method 'linear'), restated on the sorted values."""
    v = np.sort(img.reshape(-1)).astype(np.float64)
    n = v.size
    h = (n - 1) * (q / 100.0)
    lo = int(math.floor(h))
    hi = min(lo + 1, n - 1)
    t = h - lo
    a, b = v[lo], v[hi]
    d = b - a
    return float(b - d * (1.0 - t)) if t >= 0.5 else float(a + d * t)


def _cv_round(x: np.ndarray) -> np.ndarray:
    return np.rint(x)  # cvRound: round half to even (default FP rounding mode)


def area_tab(ssize: int, dsize: int):
    """computeResizeAreaTab: list per destination index of (src index, float32 alpha)."""
    scale = _cv_scale(ssize, dsize)
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        row = []
        if sx1 - fsx1 > 1e-3:
            row.append((sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            row.append((sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            row.append((sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        tab.append(row)
    return tab


def _cv_scale(ssize: int, dsize: int) -> float:
    """cv::resize's scale: 1. / inv_scale with inv_scale = (double)dsize / ssize."""
    return 1.0 / (dsize / ssize)


def resize_area_u8(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_AREA) for uint8, downscaling."""
    h, w = img.shape
    if oh == h and ow == w:
        return img.copy()
    if oh > h or ow > w:
        return resize_area_up_u8(img, oh, ow)
    sx, sy = _cv_scale(w, ow), _cv_scale(h, oh)
    eps = np.finfo(np.float64).eps
    if abs(sx - round(sx)) < eps and abs(sy - round(sy)) < eps:  # is_area_fast: resizeAreaFast_
        fx, fy = int(round(sx)), int(round(sy))
        blk = img[:oh * fy, :ow * fx].astype(np.int64).reshape(oh, fy, ow, fx).sum(axis=(1, 3))
        if fx == 2 and fy == 2:  # ResizeAreaFastVec_SIMD_8u: (a + b + c + d + 2) >> 2
            return ((blk + 2) >> 2).astype(np.uint8)
        scale = np.float32(1.0) / np.float32(fx * fy)
        return np.clip(_cv_round(blk.astype(np.float32) * scale), 0, 255).astype(np.uint8)
    xt, yt = area_tab(w, ow), area_tab(h, oh)
    out = np.empty((oh, ow), np.uint8)
    src = img.astype(np.float32)
    for dy in range(oh):
        acc = np.zeros(ow, np.float32)
        first = True
        for sy_, beta in yt[dy]:
            buf = np.zeros(ow, np.float32)
            for dx in range(ow):
                s = np.float32(0.0)
                for sx_, alpha in xt[dx]:
                    s = np.float32(s + np.float32(src[sy_, sx_] * alpha))
                buf[dx] = s
            if first:
                acc = (buf * beta).astype(np.float32)
                first = False
            else:
                acc = (acc + (buf * beta).astype(np.float32)).astype(np.float32)
        out[dy] = np.clip(_cv_round(acc), 0, 255).astype(np.uint8)
    return out


def _area_linear_coefs(ssize: int, dsize: int):
    """resizeGeneric's INTER_AREA (area_mode) linear coefficients of one axis:
    sx = floor(d * scale), f = (float)((d + 1) - (sx + 1) * inv_scale),
    f = f <= 0 ? 0 : f - floor(f); fixed point saturate_cast<short>(cbuf * 2048)
    with cbuf = {1.f - f, f} (float); 'edge' marks sx + 1 >= ssize (the
    horizontal pass then takes S[sx] * 2048, the vertical pass clips the row)."""
    inv = dsize / ssize
    scale = 1.0 / inv
    sx = np.empty(dsize, np.int64)
    c0 = np.empty(dsize, np.int64)
    c1 = np.empty(dsize, np.int64)
    for d in range(dsize):
        s = math.floor(d * scale)
        f = np.float32((d + 1) - (s + 1) * inv)
        f = np.float32(0.0) if f <= 0 else np.float32(f - np.float32(math.floor(f)))
        if s >= ssize - 1:
            s = ssize - 1
        sx[d] = s
        c0[d] = int(np.rint(np.float32(np.float32(1.0) - f) * np.float32(2048.0)))
        c1[d] = int(np.rint(f * np.float32(2048.0)))
    return sx, c0, c1


def resize_area_up_u8(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_AREA) for uint8 when
    either axis is enlarged: OpenCV (imgproc/src/resize.cpp, the generic
    non-IPP path) then runs resizeGeneric_ with area_mode coefficients
    (_area_linear_coefs) in fixed point: HResizeLinear D = S[sx] a0 + S[sx+1] a1
    (D = S[sx] * 2048 past the last full pair), VResizeLinear
    ((b0 (D0 >> 4)) >> 16) + ((b1 (D1 >> 4)) >> 16) + 2) >> 2 with rows
    clip(sy + k, 0, H-1)."""
    h, w = img.shape
    xs, a0, a1 = _area_linear_coefs(w, ow)
    ys, b0, b1 = _area_linear_coefs(h, oh)
    src = img.astype(np.int64)
    edge = xs >= w - 1
    x1 = np.minimum(xs + 1, w - 1)
    hres = np.where(edge[None, :], src[:, xs] * 2048, src[:, xs] * a0[None, :] + src[:, x1] * a1[None, :])
    r0 = hres[np.minimum(ys, h - 1)]
    r1 = hres[np.minimum(ys + 1, h - 1)]
    out = (((b0[:, None] * (r0 >> 4)) >> 16) + ((b1[:, None] * (r1 >> 4)) >> 16) + 2) >> 2
    return out.astype(np.uint8)


def resize_nearest_u8(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_NEAREST)."""
    h, w = img.shape
    ys = np.minimum(np.floor(np.arange(oh) * _cv_scale(h, oh)).astype(np.int64), h - 1)
    xs = np.minimum(np.floor(np.arange(ow) * _cv_scale(w, ow)).astype(np.int64), w - 1)
    return img[ys][:, xs]


def clahe_padding(h: int, w: int, grid: int = 8):
    """clahe.cpp: when EITHER side is not a multiple of the grid, BOTH are
    padded (bottom / right, BORDER_REFLECT_101) by grid - size % grid, so a side
    that already is a multiple gains a whole tile."""
    if h % grid or w % grid:
        return grid - h % grid, grid - w % grid
    return 0, 0


def clahe_u8(img: np.ndarray, clip_limit: float = 2.0, grid: int = 8) -> np.ndarray:
    """cv2.createCLAHE(clipLimit, (grid, grid)).apply(img) for uint8."""
    h, w = img.shape
    ph, pw = clahe_padding(h, w, grid)
    ext = np.pad(img, ((0, ph), (0, pw)), mode="reflect") if (ph or pw) else img  # BORDER_REFLECT_101
    th, tw = ext.shape[0] // grid, ext.shape[1] // grid
    area = th * tw
    limit = max(int(clip_limit * area / 256), 1) if clip_limit > 0 else 0
    lut_scale = np.float32(255.0) / np.float32(area)
    luts = np.empty((grid, grid, 256), np.uint8)
    for ty in range(grid):
        for tx in range(grid):
            tile = ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
            hist = np.bincount(tile.reshape(-1), minlength=256).astype(np.int64)
            if limit > 0:
                clipped = int(np.maximum(hist - limit, 0).sum())
                hist = np.minimum(hist, limit)
                batch = clipped // 256
                residual = clipped - batch * 256
                hist += batch
                if residual:
                    step = max(256 // residual, 1)
                    i = 0
                    while i < 256 and residual > 0:
                        hist[i] += 1
                        i += step
                        residual -= 1
            cum = np.cumsum(hist)
            luts[ty, tx] = np.clip(_cv_round(cum.astype(np.float32) * lut_scale), 0, 255).astype(np.uint8)
    inv_tw, inv_th = np.float32(1.0) / np.float32(tw), np.float32(1.0) / np.float32(th)
    xf = np.arange(w, dtype=np.float32) * inv_tw - np.float32(0.5)
    yf = np.arange(h, dtype=np.float32) * inv_th - np.float32(0.5)
    tx1 = np.floor(xf).astype(np.int64)
    ty1 = np.floor(yf).astype(np.int64)
    xa = (xf - tx1.astype(np.float32)).astype(np.float32)
    ya = (yf - ty1.astype(np.float32)).astype(np.float32)
    tx2, ty2 = np.minimum(tx1 + 1, grid - 1), np.minimum(ty1 + 1, grid - 1)
    tx1, ty1 = np.maximum(tx1, 0), np.maximum(ty1, 0)
    v = img.astype(np.int64)
    l11 = luts[ty1[:, None], tx1[None, :], v].astype(np.float32)
    l12 = luts[ty1[:, None], tx2[None, :], v].astype(np.float32)
    l21 = luts[ty2[:, None], tx1[None, :], v].astype(np.float32)
    l22 = luts[ty2[:, None], tx2[None, :], v].astype(np.float32)
    xa_, xa1 = xa[None, :], np.float32(1.0) - xa[None, :]
    ya_, ya1 = ya[:, None], np.float32(1.0) - ya[:, None]
    res = ((l11 * xa1 + l12 * xa_) * ya1 + (l21 * xa1 + l22 * xa_) * ya_).astype(np.float32)
    return np.clip(_cv_round(res), 0, 255).astype(np.uint8)


def normalize_microscopy_image(img: np.ndarray) -> np.ndarray:
    """dataset.py:30-42 on a uint8 image; float64 result as the reference's
    (np.percentile is the reference's own call; percentile_linear restates it
    for the GPU kernel and is checked against it)."""
    p_low, p_high = np.percentile(img, [2, 98])
    clipped = np.clip(img, p_low, p_high)
    c = clahe_u8(clipped.astype(np.uint8))
    return (c - c.min()) / (c.max() - c.min() + 1e-8)


def preprocess(image: np.ndarray, mask: np.ndarray, img_size=(256, 256), normalize: bool = True):
    """dataset.py:44-66 after cv2.imread: (float32 [1,h,w] image, float32 [1,h,w] mask)."""
    ow, oh = img_size  # cv2 dsize order (width, height)
    image = resize_area_u8(image, oh, ow)
    mask = resize_nearest_u8(mask, oh, ow)
    image = normalize_microscopy_image(image) if normalize else image.astype(np.float32) / np.float32(255.0)
    mask = (mask > 0).astype(np.float32)
    return image.astype(np.float32)[None], mask[None]


def rot90_vflip(img: np.ndarray, k: int, vflip: bool) -> np.ndarray:
    """A.RandomRotate90 (np.rot90(img, k)) then A.VerticalFlip (img[::-1]), dataset.py:147-151."""
    out = np.rot90(img, k)
    if vflip:
        out = out[::-1]
    return np.ascontiguousarray(out)


# ---------------------------------------------------------------------------
# CellAugmenter's interpolating transforms (dataset.py:148-154), restated from
# the published algorithms of albumentations 2.0 (A.Affine, A.AdvancedBlur;
# requirements.txt:9 pins only albumentations>=1.1.0 — 2.0.x is what pip
# resolved at the reference's snapshot) and OpenCV 4.x (cv2.warpAffine's
# fixed-point INTER_LINEAR / INTER_NEAREST path, imgproc/src/imgwarp.cpp
# WarpAffineInvoker + remapBilinear / remapNearest; cv2.filter2D's direct
# Filter2D<uchar, Cast<float, uchar>> loop).  Neither library is installed
# here: PARITY UNPINNED.  The GPU kernels (csrc/data.hip) are checked
# bit-exactly against these functions given the same sampled parameters.
# ---------------------------------------------------------------------------

def affine_matrix(scale_x: float, scale_y: float, tx_frac: float, ty_frac: float, rotate_deg: float,
                  shear_x_deg: float, shear_y_deg: float, h: int, w: int) -> np.ndarray:
    """albumentations 2.0 ``create_affine_transformation_matrix``: the FORWARD
    3x3 matrix (src -> dst) C . T . Sh . R . S . C^-1 about the image centre
    ((w-1)/2, (h-1)/2); translate is a fraction of the width / height."""
    cx, cy = (w - 1) / 2.0, (h - 1) / 2.0
    t_topleft = np.array([[1, 0, -cx], [0, 1, -cy], [0, 0, 1]], np.float64)
    s = np.array([[scale_x, 0, 0], [0, scale_y, 0], [0, 0, 1]], np.float64)
    a = np.deg2rad(rotate_deg)
    r = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]], np.float64)
    sh = np.array([[1, np.tan(np.deg2rad(shear_x_deg)), 0], [np.tan(np.deg2rad(shear_y_deg)), 1, 0], [0, 0, 1]],
                  np.float64)
    t = np.array([[1, 0, tx_frac * w], [0, 1, ty_frac * h], [0, 0, 1]], np.float64)
    t_center = np.array([[1, 0, cx], [0, 1, cy], [0, 0, 1]], np.float64)
    return t_center @ t @ sh @ r @ s @ t_topleft


def invert_affine(m) -> np.ndarray:
    """cv::invertAffineTransform on the top 2x3 rows (double), as warpAffine
    does without WARP_INVERSE_MAP: returns [M0..M5] of the dst -> src map."""
    m = np.asarray(m, np.float64).reshape(-1)[:6] if np.asarray(m).shape != (3, 3) else \
        np.asarray(m, np.float64)[:2].reshape(-1)
    d = m[0] * m[4] - m[1] * m[3]
    d = 1.0 / d if d != 0.0 else 0.0
    a11, a22 = m[4] * d, m[0] * d
    a12, a21 = -m[1] * d, -m[3] * d
    b1 = -a11 * m[2] - a12 * m[5]
    b2 = -a21 * m[2] - a22 * m[5]
    return np.array([a11, a12, b1, a21, a22, b2], np.float64)


def warp_affine_u8(img: np.ndarray, minv, nearest: bool = False) -> np.ndarray:
    """cv2.warpAffine(img, M, (w, h), flags, BORDER_CONSTANT, 0) for uint8 given
    minv = invert_affine(M): AB_BITS = 10 fixed-point source coordinates
    (cvRound of the double products), INTER_BITS = 5 sub-pixel index;
    bilinear weights (32 - f) * 32 products (initInterTab2D, exact), result
    (sum + 2^14) >> 15; taps outside the image read the border value 0, a
    pixel whose 2x2 footprint misses the image entirely is 0.  Nearest:
    (X + 512) >> 10 with the out-of-image test on the source pixel."""
    h, w = img.shape
    m = np.asarray(minv, np.float64)
    xs = np.arange(w, dtype=np.float64)
    ys = np.arange(h, dtype=np.float64)
    adelta = np.rint(m[0] * xs * 1024.0).astype(np.int64)
    bdelta = np.rint(m[3] * xs * 1024.0).astype(np.int64)
    rd = 512 if nearest else 16
    x0 = np.rint((m[1] * ys + m[2]) * 1024.0).astype(np.int64) + rd
    y0 = np.rint((m[4] * ys + m[5]) * 1024.0).astype(np.int64) + rd
    X = x0[:, None] + adelta[None, :]
    Y = y0[:, None] + bdelta[None, :]
    src = img.astype(np.int64)
    if nearest:
        sx, sy = X >> 10, Y >> 10
        inside = (sx >= 0) & (sx < w) & (sy >= 0) & (sy < h)
        out = np.where(inside, src[np.clip(sy, 0, h - 1), np.clip(sx, 0, w - 1)], 0)
        return out.astype(np.uint8)
    X, Y = X >> 5, Y >> 5
    sx, sy = X >> 5, Y >> 5
    fx, fy = X & 31, Y & 31
    w0, w1 = (32 - fy) * (32 - fx) * 32, (32 - fy) * fx * 32
    w2, w3 = fy * (32 - fx) * 32, fy * fx * 32

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
        return np.where(ok, src[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], 0)

    v = tap(sy, sx) * w0 + tap(sy, sx + 1) * w1 + tap(sy + 1, sx) * w2 + tap(sy + 1, sx + 1) * w3
    out = (v + (1 << 14)) >> 15
    miss = (sx >= w) | (sx + 1 < 0) | (sy >= h) | (sy + 1 < 0)
    return np.where(miss, 0, np.clip(out, 0, 255)).astype(np.uint8)


def advanced_blur_kernel(ksize: int, sigma_x: float, sigma_y: float, angle_deg: float, beta: float,
                         noise: np.ndarray) -> np.ndarray:
    """albumentations AdvancedBlur kernel: generalized Gaussian
    exp(-0.5 * (g^T Sigma^-1 g)^beta) on the centred ksize x ksize grid, Sigma
    = U diag(sx^2, sy^2) U^T rotated by the angle, times the multiplicative
    noise matrix, normalised to sum 1; float32 (what cv2.filter2D uses)."""
    ax = np.arange(-ksize // 2 + 1.0, ksize // 2 + 1.0)
    grid = np.stack(np.meshgrid(ax, ax), axis=-1)
    d = np.array([[sigma_x ** 2, 0], [0, sigma_y ** 2]])
    a = np.deg2rad(angle_deg)
    u = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
    inv = np.linalg.inv(u @ d @ u.T)
    k = np.exp(-0.5 * np.power(np.sum(np.dot(grid, inv) * grid, 2), beta))
    k = k * noise
    return (k.astype(np.float32) / np.sum(k)).astype(np.float32)


def filter2d_u8(img: np.ndarray, kernel: np.ndarray) -> np.ndarray:
    """cv2.filter2D(img, -1, kernel) for uint8 and an odd float32 kernel,
    anchor at the centre, BORDER_REFLECT_101: per pixel an fp32 sum over the
    NON-ZERO coefficients in row-major order, s = s + k * v (separate fp32
    multiply and add: the scalar Filter2D loop), then cvRound and saturate."""
    h, w = img.shape
    kh, kw = kernel.shape
    ry, rx = kh // 2, kw // 2
    ext = np.pad(img, ((ry, ry), (rx, rx)), mode="reflect").astype(np.float32)
    s = np.zeros((h, w), np.float32)
    for i in range(kh):
        for j in range(kw):
            f = np.float32(kernel[i, j])
            if f == 0:
                continue
            s = (s + (f * ext[i:i + h, j:j + w]).astype(np.float32)).astype(np.float32)
    return np.clip(np.rint(s), 0, 255).astype(np.uint8)
