"""Host side of CellAugmenter's interpolating transforms (dataset.py:148-154):
the per-copy parameters of ``A.Affine`` and ``A.AdvancedBlur`` turned into what
the HIP kernels (csrc/data.hip) consume — a dst -> src affine map per frame and
a float32 blur kernel per frame.  Follows albumentations 2.0's published
construction (the reference pins albumentations>=1.1.0, requirements.txt:9):

* Affine: forward matrix C . T . Sh . R . S . C^-1 about ((w-1)/2, (h-1)/2)
  (``create_affine_transformation_matrix``), inverted in double as
  cv::invertAffineTransform does inside cv2.warpAffine.
* AdvancedBlur: generalized Gaussian exp(-0.5 (g^T Sigma^-1 g)^beta) on the
  centred ksize^2 grid with Sigma = U diag(sx^2, sy^2) U^T, times the noise
  matrix, normalised, float32.
"""
from __future__ import annotations

import numpy as np


def affine_matrix(scale_x, scale_y, tx_frac, ty_frac, rotate_deg, shear_x_deg, shear_y_deg, h, w) -> np.ndarray:
    cx, cy = (w - 1) / 2.0, (h - 1) / 2.0

    def tr(dx, dy):
        return np.array([[1.0, 0.0, dx], [0.0, 1.0, dy], [0.0, 0.0, 1.0]])

    a = np.deg2rad(rotate_deg)
    rot = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
    scale = np.diag([float(scale_x), float(scale_y), 1.0])
    shear = np.array([[1.0, np.tan(np.deg2rad(shear_x_deg)), 0.0], [np.tan(np.deg2rad(shear_y_deg)), 1.0, 0.0],
                      [0.0, 0.0, 1.0]])
    return tr(cx, cy) @ tr(tx_frac * w, ty_frac * h) @ shear @ rot @ scale @ tr(-cx, -cy)


def invert_affine(m) -> np.ndarray:
    """[M0..M5] of the inverse of the top 2x3 of m (cv::invertAffineTransform)."""
    m = np.asarray(m, np.float64)[:2].reshape(-1)
    d = m[0] * m[4] - m[1] * m[3]
    d = 1.0 / d if d != 0.0 else 0.0
    a11, a22, a12, a21 = m[4] * d, m[0] * d, -m[1] * d, -m[3] * d
    return np.array([a11, a12, -a11 * m[2] - a12 * m[5], a21, a22, -a21 * m[2] - a22 * m[5]], np.float64)


def advanced_blur_kernel(ksize, sigma_x, sigma_y, angle_deg, beta, noise) -> np.ndarray:
    ax = np.arange(-ksize // 2 + 1.0, ksize // 2 + 1.0)
    grid = np.stack(np.meshgrid(ax, ax), axis=-1)
    a = np.deg2rad(angle_deg)
    u = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
    inv = np.linalg.inv(u @ np.diag([sigma_x ** 2, sigma_y ** 2]) @ u.T)
    k = np.exp(-0.5 * np.power(np.sum(np.dot(grid, inv) * grid, 2), beta)) * noise
    return (k.astype(np.float32) / np.sum(k)).astype(np.float32)
