"""lfdas — MI355X-native low-frequency DAS processing (drop-in for
DASDAE/low-freq-real-time's hot path: LFProc low-pass + decimate and the
DASCore rolling mean).  Compute runs in liblfdas.so (gfx950 HIP kernels);
this package is the host side mirroring the reference's Python surface."""
__version__ = "0.1.0"
