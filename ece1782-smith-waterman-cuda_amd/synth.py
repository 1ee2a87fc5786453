"""Deterministic synthetic protein databases.

Residues are i.i.d. from Swiss-Prot background amino-acid frequencies over
the 20 standard residues; lengths are log-normal with median 290 and mean
~360 (mu = ln 290, sigma = 0.657), clipped to [5, 35213] (the shortest and
longest Swiss-Prot entries).  Everything is a function of (seed, shard), so
any rank can regenerate any shard.  Data are synthetic: there is no network
and Swiss-Prot itself is not shipped.
"""
import numpy as np

# UniProtKB/Swiss-Prot amino-acid composition (percent), code order
# A R N D C Q E G H I L K M F P S T W Y V  (codes 0..19)
SWISSPROT_FREQ = np.array([8.25, 5.53, 4.06, 5.45, 1.37, 3.93, 6.75, 7.07, 2.27, 5.96,
                           9.66, 5.84, 2.42, 3.86, 4.70, 6.56, 5.34, 1.08, 2.92, 6.87])
LEN_MEDIAN = 290.0
LEN_SIGMA = 0.657
LEN_MIN, LEN_MAX = 5, 35213
SEED = 1782

_LUT = None


def _lut():
    """65536-entry table: uniform u16 -> residue code with the target mix."""
    global _LUT
    if _LUT is None:
        p = SWISSPROT_FREQ / SWISSPROT_FREQ.sum()
        edges = np.round(np.cumsum(p) * 65536).astype(np.int64)
        edges[-1] = 65536
        _LUT = np.searchsorted(edges, np.arange(65536), side="right").astype(np.uint8)
    return _LUT


def lengths(n, seed=SEED, shard=0, median=LEN_MEDIAN, sigma=LEN_SIGMA, lo=LEN_MIN, hi=LEN_MAX):
    rng = np.random.Generator(np.random.PCG64([seed, shard, 1]))
    L = np.exp(rng.normal(np.log(median), sigma, size=n))
    return np.clip(np.rint(L), lo, hi).astype(np.int64)


def residues(total, seed=SEED, shard=0, chunk=1 << 24):
    rng = np.random.Generator(np.random.PCG64([seed, shard, 2]))
    lut = _lut()
    out = np.empty(total, dtype=np.uint8)
    for k in range(0, total, chunk):
        m = min(chunk, total - k)
        out[k:k + m] = lut[rng.integers(0, 65536, size=m, dtype=np.uint16)]
    return out


def database(n, seed=SEED, shard=0, **len_kw):
    """(residues uint8, offsets int64[n+1]) for a synthetic shard."""
    L = lengths(n, seed, shard, **len_kw)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(L)
    return residues(int(offs[-1]), seed, shard), offs


def fixed_length_database(n, mean, sd, seed=SEED, shard=0, lo=1):
    """Normal lengths N(mean, sd) (config C5: 2k-residue subjects)."""
    rng = np.random.Generator(np.random.PCG64([seed, shard, 3]))
    L = np.clip(np.rint(rng.normal(mean, sd, size=n)), lo, None).astype(np.int64)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(L)
    return residues(int(offs[-1]), seed, shard), offs


def query(length, seed=SEED, shard=99):
    return residues(length, seed, shard)


# ---------------------------------------------------------------------------
# Counter-based generator: a pure-numpy restatement
# of the library's on-device generator (sw_db_create_synthetic, sw_synth.hip),
# so any sampled subject of a device-generated shard can be regenerated on a
# CPU.  Integer-only; the two tables come from the library (sw_synth_tables).
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1
LEN_SALT = 0x4C454E475448


def _mix(z):
    """splitmix64's finaliser (arithmetic mod 2^64)."""
    with np.errstate(over="ignore"):
        z = np.asarray(z, dtype=np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def counter_hash(seed, ids, k):
    """h(seed, id, k) = mix(seed * G1 + mix(id * G2 + k)) mod 2^64."""
    with np.errstate(over="ignore"):
        ids = np.asarray(ids, dtype=np.uint64)
        k = np.asarray(k, dtype=np.uint64)
        inner = _mix(ids * np.uint64(0xD6E8FEB86659FD93) + k)
        return _mix(np.uint64((seed * 0x9E3779B97F4A7C15) & _M64) + inner)


def counter_lengths(seed, gids, len_table):
    h = counter_hash(seed, gids, LEN_SALT)
    return len_table[(h >> np.uint64(52)).astype(np.int64)]


def counter_residues(seed, gid, length, lut):
    """Residue codes of global subject `gid` (length from counter_lengths)."""
    words = (length + 3) // 4
    h = counter_hash(seed, np.full(words, gid, dtype=np.uint64), np.arange(words, dtype=np.uint64))
    parts = [(h >> np.uint64(16 * e)) & np.uint64(0xFFFF) for e in range(4)]
    idx = np.stack(parts, axis=1).reshape(-1)[:length].astype(np.int64)
    return lut[idx]
