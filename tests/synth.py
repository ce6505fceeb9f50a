"""Synthetic segments for parity tests (seeded, small enough for the oracle to finish in seconds)."""
import numpy as np

from pinot_amd.segment import create_segment


def make_values(rng, n, dtype, card, skew=False):
    if dtype == "STRING":
        pool = np.array(["s%05d_%s" % (i, "x" * (i % 7)) for i in range(card)])
        idx = rng.zipf(1.3, size=n) % card if skew else rng.integers(0, card, size=n)
        return pool[idx]
    if dtype in ("INT", "LONG"):
        span = (1 << 31) - 1 if dtype == "INT" else (1 << 33)  # sums stay < 2^53
        pool = np.unique(rng.integers(-span // 4, span, size=card * 2))[:card]
        if dtype == "INT":
            pool = pool.astype(np.int32)
    else:
        pool = np.unique(np.round(rng.normal(0, 1e4, size=card * 2), 3))[:card]
        if dtype == "FLOAT":
            pool = np.unique(pool.astype(np.float32))
    idx = rng.zipf(1.3, size=n) % len(pool) if skew else rng.integers(0, len(pool), size=n)
    return pool[idx]


def make_segment(seed, n, columns, name=None, no_dict=()):
    """columns: {name: (dtype, cardinality)}; raw (no-dict) columns draw random values of the dtype."""
    rng = np.random.default_rng(seed)
    data, schema = {}, {}
    for c, (dt, card) in columns.items():
        schema[c] = dt
        if c in no_dict:
            if dt in ("INT", "LONG"):
                data[c] = rng.integers(-1000, 1000, size=n).astype(np.int32 if dt == "INT" else np.int64)
            else:
                data[c] = rng.normal(0, 100, size=n).astype(np.float32 if dt == "FLOAT" else np.float64)
        else:
            data[c] = make_values(rng, n, dt, card, skew=(seed % 2 == 1))
    return create_segment(name or "seg%d" % seed, data, schema, no_dictionary_columns=no_dict)
