"""Reduction of a measured FR to fewer frequencies (``source/jax_plate/Input.py``).

``Compressor(freqs, complex_fr, max_size, use_alg)(desired_size)`` keeps the
reference's two algorithms and their outputs (pinned by
``tests/golden/compressor.npz``, generated from the reference class):

* ``use_alg=0``: every ``size/desired_size``-th sample (float stride, index 0
  dropped if the stride overshoots);
* ``use_alg=1``: peaks and troughs of the Savitzky-Golay-smoothed log-amplitude
  (distance ~75 Hz, width > 20 samples, prominence > 0.1, smoothness < 50), a
  symmetric window around each, then windows grown one sample at a time until
  ``desired_size`` samples are selected.
"""
from __future__ import annotations

import numpy as np
from scipy.signal import find_peaks, peak_prominences, peak_widths, savgol_filter


class Compressor:
    def __init__(self, freqs: np.ndarray, complex_fr: np.ndarray, max_size: int, use_alg: int):
        assert freqs.size == complex_fr.size
        self.size = freqs.size
        self.freqs = freqs
        self.complex_fr = complex_fr
        self.max_size = max_size
        self.alg = use_alg

    @staticmethod
    def _peak_smoothness(x: np.ndarray, peaks: np.ndarray) -> np.ndarray:
        """Inverse mean absolute increment over +-10 neighbours (scaled to 20 steps)."""
        out = np.empty(peaks.size, dtype=np.float64)
        for k, p in enumerate(peaks):
            half = 10 if (p > 10 and x.size - p > 10) else min(p, x.size - p) - 1
            seg = x[p - half:p + half + 1]
            out[k] = np.abs(np.diff(seg)).sum() * 10.0 / half
        return 1.0 / out

    def _uniform(self, n: int) -> np.ndarray:
        mask = np.zeros(self.size, dtype=bool)
        stride = self.size / n
        pos = 0.0
        while pos < self.size:
            mask[int(pos)] = True
            pos += stride
        if mask.sum() > n:
            mask[0] = False
        return mask

    def _peaks(self, n: int) -> np.ndarray:
        mask = np.zeros(self.size, dtype=bool)
        dist = int(75 / np.max(np.diff(self.freqs)))
        la = np.log(savgol_filter(np.abs(self.complex_fr), 30, 3))
        found = []
        for sig in (la, -la):
            pk = find_peaks(sig, distance=dist)[0]
            pk = pk[peak_widths(sig, pk)[0] > 20]
            pk = pk[peak_prominences(sig, pk)[0] > 0.1]
            found.append(pk[self._peak_smoothness(sig, pk) < 50])
        idx = np.concatenate(found)
        npk = idx.size
        layers = (n - npk) // (npk * 2)
        lo = np.maximum(idx - layers, 0)
        hi = idx + layers
        hi[hi + 1 > self.size] = self.size
        for a, b in zip(lo, hi):
            mask[a:b + 1] = True
        missing = n - mask.sum()
        while missing != 0:
            for k in range(npk - 1):
                if hi[k] < lo[k + 1]:
                    hi[k] += 1
                    missing -= 1
                    mask[hi[k] + 1] = True
                if missing == 0:
                    break
            if missing == 0:
                break
            if hi[-1] + 1 < self.size:
                hi[-1] += 1
                missing -= 1
                mask[hi[-1]] = True
            elif lo[0] - 1 > 0:
                lo[0] -= 1
                missing -= 1
                mask[lo[0]] = True
        return mask

    def __call__(self, desired_size: int):
        if desired_size > self.max_size:
            raise ValueError(f'Desired size of compressed data must be lower than {self.max_size + 1}')
        if self.alg == 0:
            mask = self._uniform(desired_size)
        elif self.alg == 1:
            mask = self._peaks(desired_size)
        else:
            mask = np.zeros(self.size, dtype=bool)
        return self.freqs[mask], self.complex_fr[mask]
