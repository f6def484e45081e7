"""Post-processing of the decimated output on device — the numpy/scipy steps
the reference notebooks run on ``LFProc``'s results
(low_pass_dascore.ipynb cells 14-22):

* ``scale_iDAS(sampling_rate, gauge_length)`` — ``(116*fs/gauge)/1e9``
  (strain-rate scale, cells 14/18/22);
* ``demean_scale(data, c0, c1, scale)`` — ``(data - mean(data[:, c0:c1],
  axis=1)[:, None]) * scale`` on (time, distance) data (cells 14/18/22);
* ``median_filter(a, size)`` — ``scipy.ndimage.median_filter(a, size=size)``
  (mode 'reflect', cells 16/20), 1-D traces or 2-D arrays.

Inputs are float64 numpy arrays (returned as numpy) or CUDA tensors
(returned as CUDA tensors); the work runs in liblfdas.so
(``lfd_demean_scale_f64``, ``lfd_median_filter_f64``)."""
from __future__ import annotations

import numpy as np

from ._lib import check, load


def scale_iDAS(sampling_rate: float, gauge_length: float) -> float:
    """low_pass_dascore.ipynb cell 14: ``float((116*sampling_rate/gauge_length)/1e9)``."""
    return float((116 * sampling_rate / gauge_length) / 1e9)


def _to_dev(a):
    import torch
    if isinstance(a, torch.Tensor):
        if not a.is_cuda:
            raise TypeError("tensor inputs must be on the HIP device")
        return a.to(torch.float64), True
    if not torch.cuda.is_available():
        raise RuntimeError("lfdas needs a HIP device (MI355X); no CPU fallback")
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda(), False


def _stream():
    import torch
    return int(torch.cuda.current_stream().cuda_stream)


def demean_scale(data, ch_start: int, ch_end: int, scale: float = 1.0):
    """``(data - mean(data[:, ch_start:ch_end], axis=1)[:, None]) * scale`` for
    (time, distance) data (one mean per time sample over the channel range)."""
    import torch
    x, was_t = _to_dev(data)
    if x.dim() != 2:
        raise ValueError("demean_scale takes 2-D (time, distance) data")
    y = torch.empty_like(x, memory_format=torch.contiguous_format)
    check(load().lfd_demean_scale_f64(x.data_ptr(), x.shape[0], x.shape[1], x.stride(0), x.stride(1),
                                      int(ch_start), int(ch_end), float(scale), y.data_ptr(),
                                      y.stride(0), y.stride(1), _stream()))
    return y if was_t else y.cpu().numpy()


def median_filter(a, size):
    """``scipy.ndimage.median_filter(a, size=size)`` (mode 'reflect', origin
    0) for 1-D or 2-D float64 data; ``size`` an int or a per-axis tuple."""
    import torch
    x, was_t = _to_dev(a)
    one_d = x.dim() == 1
    if one_d:
        x = x[None, :]
    if x.dim() != 2:
        raise ValueError("median_filter takes 1-D or 2-D data")
    if np.ndim(size) == 0:
        k = (1, int(size)) if one_d else (int(size), int(size))
    else:
        k = tuple(int(v) for v in size)
        if one_d:
            k = (1,) + k
    if len(k) != 2:
        raise ValueError("size must have one entry per axis")
    if one_d and k[1] > 2 * x.shape[1]:
        # scipy's 1-D rank filter extends such lines differently from its
        # n-D path; not restated
        raise NotImplementedError("1-D median window longer than twice the trace")
    y = torch.empty(tuple(x.shape), dtype=torch.float64, device=x.device)
    check(load().lfd_median_filter_f64(x.data_ptr(), x.shape[0], x.shape[1], x.stride(0), x.stride(1),
                                       k[0], k[1], y.data_ptr(), y.stride(0), y.stride(1), _stream()))
    if one_d:
        y = y[0]
    return y if was_t else y.cpu().numpy()
