"""The bin stepper's instance rule on the CPU: ecdna_ssa_ctx_create picks the instruction
schedule / lane pairing through bin_schedule_rule (ecdna-evo_amd/csrc/ssa_api.cpp), a pure function of the run's shape
and the two builds' occupancies, exported for these tests as ecdna_dev_bin_schedule (not part of the C ABI). Here every
bench shape is walked through it with the occupancies its instance reports on the GPU (tests/test_gpu_bench_instances.py
asserts the same choices on hardware), and the rule's invariants are checked over a grid of user shapes."""
import ctypes as C
import itertools
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "ecdna-evo_amd", "lib", "libecdna_ssa.so")
CUS, BLOCK = 256, 256
AUTO = 2


@pytest.fixture(scope="module")
def rule():
    if not os.path.exists(LIB):
        import __graft_entry__

        __graft_entry__.build()
    fn = C.CDLL(LIB).ecdna_dev_bin_schedule
    fn.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int,
                   C.c_uint32]
    fn.restype = C.c_int

    def call(max_chunk, pair_ok=True, k64u16=False, tf0=True, occ_def=4, occ_ilp=4, pair_mode=AUTO, sched=AUTO):
        return fn(int(pair_ok), pair_mode, sched, max_chunk, CUS, int(k64u16), int(tf0), occ_def, occ_ilp, BLOCK)

    return call


# (shape, replicates in the largest chunk, rule inputs, schedule the bench instance reports)
BENCH = [
    ("C3, 2^20 per GPU (K = 32 / u32; both builds 4 workgroups per CU)", 1 << 20, {}, 1),
    ("C3 fixed total, 8-GPU shard", 1 << 17, {}, 1),
    ("C2 (pure birth: no pairing)", 65_536, {"pair_ok": False}, 1),
    ("C5, 8-GPU shard: half a wave per SIMD, paired", 32_768, {}, 3),
    ("C5, 4-GPU shard: one wave per SIMD", 65_536, {}, 1),
    ("C5 whole (K = 64 / u32: LDS bounds both builds at 2 workgroups per CU)", 262_144, {"occ_def": 2, "occ_ilp": 2}, 1),
    ("C4, 8-GPU shard (K = 64 / u16: default 4, max-ILP 3 workgroups per CU; 2 per lane)", 524_288,
     {"k64u16": True, "occ_def": 4, "occ_ilp": 3}, 1),
    ("C4 whole (16 per lane): the 128-VGPR build", 4_194_304, {"k64u16": True, "occ_def": 4, "occ_ilp": 3}, 2),
    ("C4 whole with f32 time and the hash (the 128-VGPR build spills there)", 4_194_304,
     {"k64u16": True, "tf0": False, "occ_def": 4, "occ_ilp": 3}, 0),
]


@pytest.mark.parametrize("name,n,kw,expect", BENCH, ids=[b[0].split(",")[0] + f"-{b[1]}" for b in BENCH])
def test_bench_shapes_choose_their_instances(rule, name, n, kw, expect):
    assert rule(n, **kw) == expect, name


def test_overrides(rule):
    assert rule(1 << 20, pair_mode=3) == 1  # (round 5's quads, ECDNA_SSA_PAIR = 3, are gone: 3 is auto-like, unpaired)
    assert rule(1 << 20, pair_ok=False, pair_mode=1) == 1  # (no pairs without a paired instance)
    assert rule(32_768, pair_mode=0) == 1  # pairing off
    assert rule(1 << 20, pair_mode=1) == 3  # pairs forced
    assert rule(32_768, sched=0) == 0 and rule(1 << 20, sched=1) == 1
    assert rule(1 << 20, sched=3, k64u16=True) == 2 and rule(1 << 20, sched=3) == 0


@pytest.mark.parametrize("pair_ok,k64u16,tf0", list(itertools.product([False, True], repeat=3)))
def test_rule_invariants_over_user_shapes(rule, pair_ok, k64u16, tf0):
    """pairs only with a paired instance and at most half a wave of replicates per SIMD; the
    128-VGPR build only for K = 64 / u16 without the runtime-flag variant; one wave per SIMD or less is max-ILP"""
    for n, (od, oi) in itertools.product([1, 100, 32_768, 32_769, 65_536, 65_537, 1 << 20, 1 << 22, 1 << 24],
                                         [(4, 4), (4, 3), (3, 4), (2, 2)]):
        s = rule(n, pair_ok=pair_ok, k64u16=k64u16, tf0=tf0, occ_def=od, occ_ilp=oi)
        assert s in (0, 1, 2, 3)
        assert (s == 3) == (pair_ok and n <= CUS * BLOCK // 2)
        if s == 2:
            assert k64u16 and tf0
        if n <= CUS * BLOCK and s != 3:
            assert s == 1
