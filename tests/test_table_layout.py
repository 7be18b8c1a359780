"""Feature table layout (CPU, no GPU): the "primary first" cuckoo table built by
lt_image_build (lt_capi.cpp cuckoo_build) answers every key with the lookup the
kernels do (lt_decode.hip probe_issue / probe_finish): load the primary slot;
on a miss at a flagged slot load the secondary.  Absent keys are never found.

The slot hash is restated here in numpy from lt_common.h (narrow_hash,
narrow_slot1/2) -- an independent check of the layout the device relies on.
"""
import numpy as np
import pytest

from lattice_based_tagger_amd import _capi, synth

M32 = np.uint64(0xFFFFFFFF)
FLAG = np.uint64(1) << np.uint64(63)


def _u32(x):
    return np.asarray(x, dtype=np.uint64) & M32


def narrow_hash(seed):
    x, v = seed, []
    for i in range(8):
        x = (x * 0x9E3779B1 + 0x7F4A7C15) & 0xFFFFFFFF
        y = x ^ (x >> 15)
        y = (y * 0x2C1B3C6D) & 0xFFFFFFFF
        y ^= y >> 12
        y = (y * 0x297A2D39) & 0xFFFFFFFF
        y ^= y >> 15
        v.append((y | 1) if i in (3, 4, 7) else ((y & 0xFFFFFF) | 0x800001))
    return v


def mul24(x, k):
    return _u32((np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFF)) * np.uint64(k & 0xFFFFFF))


def slot(h, a, b, c, cls, slots, which):
    """HASH_VERSION 5: one mix x over the key without its sub component (the
    tag of classes 0 / 1 / 2 / 3: c, b, a, b), i1 = (x >> s) & ~15 | sub & 15
    (x >> s for classes 7 / 8), i2 = ((x ^ x >> 16 ^ sub) * K2) >> s on 2^n
    slots (s = 32 - n)."""
    assert slots & (slots - 1) == 0
    shift = np.uint64(32 - (int(slots).bit_length() - 1))
    cls = np.asarray(cls)
    sp = np.select([cls == 0, cls == 1, cls == 2, cls == 3], [2, 1, 0, 1], -1)
    comps = [np.asarray(a, np.uint64), np.asarray(b, np.uint64), np.asarray(c, np.uint64)]
    zero = np.uint64(0)
    ma, mb, mc = (np.where(sp == i, zero, mul24(comps[i], h[i])) for i in range(3))
    sub = np.select([sp == 0, sp == 1, sp == 2], comps, zero).astype(np.uint64)
    x = ma ^ mb ^ mc ^ _u32(cls.astype(np.uint64) * np.uint64(h[3]))
    if which == 2:
        return (_u32((x ^ (x >> np.uint64(16)) ^ sub) * np.uint64(h[4])) >> shift).astype(np.int64)
    i = x >> shift
    g = np.uint64(15)
    return np.where(sp >= 0, (i & ~g) | (sub & g), i).astype(np.int64)


def narrow_key(a, b, c, cls):
    code = np.where(cls == 8, 4, cls).astype(np.uint64)
    return (code << np.uint64(60)) | (a.astype(np.uint64) << np.uint64(40)) | \
        (b.astype(np.uint64) << np.uint64(20)) | c.astype(np.uint64)


def lookup(table, h, slots, a, b, c, cls):
    """The device lookup over arrays of keys: (found, coef, slot loads)."""
    key = narrow_key(a, b, c, cls)
    tk = table[:, 0]
    i1 = slot(h, a, b, c, cls, slots, 1)
    s1 = tk[i1]
    hit1 = (s1 & ~FLAG) == key
    need2 = ~hit1 & ((s1 & FLAG) != 0)
    i2 = slot(h, a, b, c, cls, slots, 2)
    hit2 = need2 & ((tk[i2] & ~FLAG) == key)
    coef = np.where(hit1, table[i1, 1], table[i2, 1]).view(np.float64)
    return hit1 | hit2, coef, 1 + need2.astype(np.int64)


@pytest.fixture(scope='module')
def model():
    raw = synth.make_lattices(2048, seed=5)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=5, n_features=200_000)
    _, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    img = _capi.ModelImage(keys, coefs)
    arr = img.arrays()
    img.close()
    return keys.reshape(-1, 4).astype(np.int64), coefs, arr


def test_every_key_found_with_primary_first_lookup(model):
    keys, coefs, arr = model
    assert arr['narrow'] == 1 and arr['hash_version'] == 5
    table = arr['table'].view(np.uint64).reshape(-1, 2)
    h = narrow_hash(arr['seed'])
    a, b, c, cls = keys.T
    found, coef, loads = lookup(table, h, arr['slots'], a, b, c, cls)
    assert found.all()
    assert np.array_equal(coef.view(np.uint64), coefs.view(np.uint64))
    # most keys sit at their primary slot: one load
    assert loads.mean() < 1.3
    # each key is stored exactly once
    occupied = (table[:, 0] & ~FLAG) != 0
    assert int(occupied.sum()) == len(keys)


def test_absent_keys_not_found(model):
    keys, _, arr = model
    table = arr['table'].view(np.uint64).reshape(-1, 2)
    h = narrow_hash(arr['seed'])
    rng = np.random.default_rng(0)
    n = 200_000
    a, b, c, cls = keys[rng.integers(0, len(keys), n)].T.copy()
    # perturb one component so the key is (almost surely) absent
    c = np.where(c > 0, c + 1 + rng.integers(0, 1000, n), 0)
    b = np.where(c == 0, b + 1 + rng.integers(0, 1000, n), b)
    present = set(map(tuple, keys.tolist()))
    absent = np.array([tuple(x) not in present for x in zip(a.tolist(), b.tolist(), c.tolist(), cls.tolist())])
    found, _, loads = lookup(table, h, arr['slots'], a, b, c, cls)
    assert not found[absent].any()
    assert loads[absent].mean() < 1.2          # a second load only at flagged primaries
