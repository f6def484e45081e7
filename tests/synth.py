"""Seeded synthetic inputs shared by the golden-fixture generator and tests
(no dataset exists; DASCore's random_das convention for cfg1)."""
import numpy as np

T0_NS = 1_505_692_800_000_000_000  # 2017-09-18T00:00:00


def random_das_spool_data(n_patches=3, shape=(300, 2000)):
    """DASCore get_example_spool('random_das') data: each patch is
    RandomState(42).random(shape) (float64), patches concatenated in time."""
    return np.concatenate([np.random.RandomState(42).random(shape)] * n_patches, axis=1)


def noise_sine(n_ch, n, fs, seed, dc=0.0, f0=0.05):
    """0.5-amplitude sine + N(0,1) (+ dc), float32."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    phi = rng.random((n_ch, 1)) * 2 * np.pi
    return (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * f0 * t + phi) + dc).astype(np.float32)


def digest(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
