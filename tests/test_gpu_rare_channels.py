"""Rare channels on the GPU (draw mapping v7): the engine fires a channel of probability ~1e-6 exactly on
the words where the oracle does, and then continues the same trajectory.

tests/test_mapping_v7.py proves, on the oracle's channel function, that every channel's probability is within 2^-32 of
lambda_i / sum(lambda). Here the GPU is held to that function at states where a channel is rare: one N- cell among
10^6 N+ cells (pure birth b0 = b1 = 1: ProliferateNMinus w.p. 1/(10^6 + 1); birth-death at C3's rates: ProliferateNMinus
and DeathNMinus w.p. 1 / 1.8e6 and 0.3 / 1.8e6). The replicate ids whose first event draws the rare channel are found on
the CPU (Philox4x32-10 over 2^25 ids, confirmed with oracle_channel); each runs on the GPU (row and bin stores) for one
event and for 64 events, bit for bit against the oracle. Under v6 (23-bit channel uniform) the pure-birth channel
had 8 2^-23 instead of 1/(10^6 + 1) (-4.6 %)."""
import dataclasses
import functools

import numpy as np
import pytest

from ecdna_evo_amd import abi

SEED = 42
M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def _philox_w1(rids, seed):
    """word 1 of Philox4x32-10((e = 0, 0, rid lo, rid hi), (seed lo, seed hi)) for every id (numpy, vectorised)"""
    rids = rids.astype(np.uint64)
    c0 = np.zeros_like(rids)
    c1 = np.zeros_like(rids)
    c2 = rids & MASK
    c3 = rids >> np.uint64(32)
    k0, k1 = seed & 0xFFFFFFFF, seed >> 32
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = np.uint64(M0) * c0
        p1 = np.uint64(M1) * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0), p1 & MASK,
                          (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1), p0 & MASK)
    return c1.astype(np.uint32)


def test_numpy_philox_matches_oracle(oracle_mod):
    ids = np.array([0, 1, 12345, (1 << 32) + 7], dtype=np.uint64)
    w1 = _philox_w1(ids, SEED)
    for rid, w in zip(ids.tolist(), w1.tolist()):
        out = oracle_mod.philox((0, 0, rid & 0xFFFFFFFF, rid >> 32), (SEED & 0xFFFFFFFF, SEED >> 32))
        assert out[1] == w


STATES = {  # name: (process, rates, rare channels)
    "pure_birth": (abi.PURE_BIRTH, (1.0, 1.0, 0.0, 0.0), (abi.EV_PROLIF_NMINUS,)),
    "birth_death": (abi.BIRTH_DEATH, (1.0, 1.5, 0.3, 0.3), (abi.EV_PROLIF_NMINUS, abi.EV_DEATH_NMINUS)),
}
NPLUS = 1_000_000


def _first_word(oracle_mod, rates, bd, i):
    """the first word w1 drawing a channel >= i from (1 N- cell, NPLUS N+ cells): the channel is non-decreasing in w1"""
    lo, hi = 0, 1 << 32
    while lo < hi:
        mid = (lo + hi) // 2
        if oracle_mod.channel(rates, 1, NPLUS, bd, mid) >= i:
            hi = mid
        else:
            lo = mid + 1
    return lo


@functools.lru_cache(maxsize=None)
def _rare_ids(oracle_mod, process, rates, channels, n_ids=1 << 25, chunk=1 << 22):
    """ids < n_ids whose event-0 word w1 draws one of `channels`, per channel"""
    bd = process == abi.BIRTH_DEATH
    win = {ch: ((_first_word(oracle_mod, rates, bd, ch) if ch else 0), _first_word(oracle_mod, rates, bd, ch + 1))
           for ch in channels}
    out = {ch: [] for ch in channels}
    for start in range(0, n_ids, chunk):
        w1 = _philox_w1(np.arange(start, start + chunk, dtype=np.uint64), SEED).astype(np.uint64)
        for ch, (lo, hi) in win.items():
            for r in np.nonzero((w1 >= lo) & (w1 < hi))[0].tolist():
                assert oracle_mod.channel(rates, 1, NPLUS, bd, int(w1[r])) == ch
                out[ch].append(start + r)
    return out


@pytest.mark.parametrize("state", sorted(STATES))
def test_rare_ids_exist(oracle_mod, state):
    """ids draw each rare channel at event 0 for the GPU test (2^25 / 1.8e6 ~ 19 for ProliferateNMinus, ~ 5.6 for
    DeathNMinus)"""
    process, rates, channels = STATES[state]
    ids = _rare_ids(oracle_mod, process, rates, channels)
    for ch in channels:
        assert len(ids.get(ch, [])) >= 1, ids


@pytest.mark.gpu
@pytest.mark.parametrize("store", ["rows", "bins"])
@pytest.mark.parametrize("state", sorted(STATES))
def test_gpu_rare_channel_fires_where_the_oracle_does(engine_mod, oracle_mod, state, store):
    process, rates, channels = STATES[state]
    ids = _rare_ids(oracle_mod, process, rates, channels)
    flags = abi.FLAG_EVENT_HASH | (abi.FLAG_BIN_STORE if store == "bins" else 0)
    for ch, rids in sorted(ids.items()):
        for rid in rids[:3]:
            base = abi.RunSpec(seed=SEED, process=process, rates=(rates,), reps_per_set=1 << 40, first_replicate=rid,
                               n_replicates=1, max_cells=NPLUS + 10_000, init={0: 1, 1: NPLUS}, flags=flags,
                               bin_kmax=32 if store == "bins" else 0, hist_bins=64)
            for iters in (1, 64):
                spec = dataclasses.replace(base, max_iter=iters, _keep=[])
                gpu = engine_mod.run(spec, want_rows=True)
                cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
                for f in gpu.summaries.dtype.names:
                    a, b = gpu.summaries[f], cpu.summaries[f]
                    if f == "time":
                        a, b = a.view(np.uint64), b.view(np.uint64)
                    np.testing.assert_array_equal(a, b, err_msg=f"{state}/{store} rid {rid} iters {iters}: {f}")
                np.testing.assert_array_equal(gpu.row(0), cpu.row(0))
                np.testing.assert_array_equal(gpu.hist, cpu.hist)
                if iters == 1:  # the one event drawn is the rare channel
                    assert int(gpu.summaries["events_by_type"][0][ch]) == 1, (rid, gpu.summaries["events_by_type"])
