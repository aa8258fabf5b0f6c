"""Parity cases shared by the GPU parity tests and the golden-fixture generator.

Each case is a small RunSpec the CPU oracle finishes in well under a second. Together they cover
both processes, all four segregation rules, f32/f64 time, the birth-death cap-compat flag, single-
and multi-set (ABC) runs, non-default initial distributions, replicate-id offsets and strides (sharding) and
every stop reason and per-replicate error the engine reports.

bin_cases() runs the same cases through the bin store (ECDNA_FLAG_BIN_STORE), plus
cases aimed at its boundaries: copy numbers around bin_kmax (daughters crossing it, picks from the
large-k row, swap_remove inside it), the 256-bin variant and u32 counters (cell_cap > 65535).
"""
import dataclasses

from ecdna_evo_amd import abi

H = abi.FLAG_EVENT_HASH

BD_RATES = ((1.0, 1.5, 0.3, 0.3),)  # C3 shape


def cases():
    c = {}
    # C1 shape: pure birth + binomial to 1e3 cells, seed 42 (BASELINE.json configs[0])
    c["pb_binomial_c1"] = abi.RunSpec(seed=42, n_replicates=64, max_cells=1000, flags=H)
    for name, seg in abi.SEGREGATION_NAMES.items():
        c[f"pb_{name}"] = abi.RunSpec(seed=7, segregation=seg, n_replicates=48, max_cells=600,
                                      init={3: 2, 8: 1}, flags=H)
        c[f"bd_{name}"] = abi.RunSpec(seed=11, segregation=seg, process=abi.BIRTH_DEATH, rates=BD_RATES,
                                      n_replicates=48, max_cells=800, flags=H)
    c["pb_f32_time"] = abi.RunSpec(seed=5, n_replicates=32, max_cells=500, flags=H | abi.FLAG_TIME_F32)
    c["bd_f32_time"] = abi.RunSpec(seed=5, process=abi.BIRTH_DEATH, rates=BD_RATES, n_replicates=32,
                                   max_cells=500, flags=H | abi.FLAG_TIME_F32)
    c["bd_cap_compat"] = abi.RunSpec(seed=9, process=abi.BIRTH_DEATH, rates=BD_RATES, n_replicates=32,
                                     max_cells=1000, flags=H | abi.FLAG_BD_CAP_COMPAT)
    c["bd_selection"] = abi.RunSpec(seed=3, process=abi.BIRTH_DEATH, rates=((1.0, 2.0, 0.5, 0.1),),
                                    n_replicates=32, max_cells=1500, init={1: 4, 0: 2}, flags=H)
    # turnover: d close to b, 1000 initial cells, time-capped (C5 shape, scaled down)
    c["bd_turnover"] = abi.RunSpec(seed=13, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),),
                                   n_replicates=16, max_cells=1_300, max_time=3.0, init={1: 1000}, flags=H)
    # shrinking populations: N+ deaths walk the LDS tail window down through many 16-cell blocks
    c["bd_shrink"] = abi.RunSpec(seed=19, process=abi.BIRTH_DEATH, rates=((1.0, 0.6, 0.2, 1.4),), n_replicates=32,
                                 max_cells=5000, init={1: 150, 2: 60, 9: 37}, flags=H)
    c["bd_oscillate"] = abi.RunSpec(seed=23, process=abi.BIRTH_DEATH, rates=((0.5, 1.0, 0.5, 1.0),),
                                    n_replicates=32, max_cells=100, max_time=40.0, init={3: 33}, flags=H)
    # extinction-prone: death > birth -> Absorbing
    c["bd_extinction"] = abi.RunSpec(seed=17, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 1.5, 1.5),),
                                     n_replicates=64, max_cells=400, init={2: 3}, flags=H)
    # ABC shape: 4 parameter sets x 8 replicates, per-set initial distributions (C4, scaled down)
    c["abc_sets"] = abi.RunSpec(
        seed=42, process=abi.BIRTH_DEATH, segregation=abi.SEG_BINOMIAL,
        rates=((1.0, 1.0, 0.1, 0.1), (1.0, 1.5, 0.1, 0.1), (1.0, 2.0, 0.3, 0.2), (1.0, 2.5, 0.0, 0.4)),
        reps_per_set=8, n_replicates=32, max_cells=700, hist_bins=257,
        init_per_set=[{1: 1}, {2: 1}, {4: 1, 0: 3}, {8: 2}], flags=H)
    # replicate-id offset: a shard of a bigger run
    c["shard_offset"] = abi.RunSpec(seed=42, first_replicate=1000, n_replicates=40, max_cells=700,
                                    reps_per_set=100000, flags=H)
    # interleaved shards (replicate_stride): ids 3, 8, ..., 198 of one set; ids 1, 4, ..., 31 across the 4 ABC sets
    c["shard_interleaved"] = abi.RunSpec(seed=42, first_replicate=3, replicate_stride=5, n_replicates=40,
                                         max_cells=700, reps_per_set=100000, flags=H)
    c["abc_sets_interleaved"] = dataclasses.replace(c["abc_sets"], first_replicate=1, replicate_stride=3,
                                                    n_replicates=11, _keep=[])
    # large copy numbers: n = 2k > 32 takes the multi-block popcount path
    c["big_copies"] = abi.RunSpec(seed=21, n_replicates=24, max_cells=300, init={40: 2, 300: 1, 5000: 1},
                                  hist_bins=64, flags=H)
    c["big_copies_no_uneven"] = abi.RunSpec(seed=22, segregation=abi.SEG_BINOMIAL_NO_UNEVEN, n_replicates=24,
                                            max_cells=300, init={17: 2, 64: 1}, flags=H)
    # copy numbers 17..48: segregation draws from w3 plus the spare words of earlier events (draw mapping
    # v3), with birth-death and N- events refilling the spares, and NoUneven redraws on top of them
    c["spares_mid_copies"] = abi.RunSpec(seed=51, process=abi.BIRTH_DEATH, rates=((0.8, 1.2, 0.5, 0.4),),
                                         n_replicates=32, max_cells=900, init={20: 30, 31: 10, 33: 5, 0: 20},
                                         hist_bins=128, flags=H)
    c["spares_no_uneven"] = abi.RunSpec(seed=52, segregation=abi.SEG_BINOMIAL_NO_UNEVEN, n_replicates=24,
                                        max_cells=500, init={17: 4, 24: 4, 32: 2, 1: 6}, hist_bins=128, flags=H)
    # stop reasons and errors
    c["max_iter"] = abi.RunSpec(seed=1, n_replicates=16, max_cells=10_000, max_iter=137, flags=H)
    c["max_time"] = abi.RunSpec(seed=2, n_replicates=16, max_cells=100_000, max_time=2.5, cell_cap=4096, flags=H)
    c["overflow"] = abi.RunSpec(seed=3, n_replicates=8, max_cells=50, init={32768: 1, 1: 1}, flags=H)
    c["no_overflow_edge"] = abi.RunSpec(seed=3, segregation=abi.SEG_DETERMINISTIC, n_replicates=8, max_cells=50,
                                        init={32767: 1}, flags=H)
    c["cell_cap_error"] = abi.RunSpec(seed=4, n_replicates=8, max_cells=5000, cell_cap=100, flags=H)
    c["empty_init"] = abi.RunSpec(seed=5, n_replicates=4, max_cells=100, init={}, flags=H)
    c["nminus_only"] = abi.RunSpec(seed=6, n_replicates=4, max_cells=100, init={0: 5}, flags=H)
    c["already_full"] = abi.RunSpec(seed=6, n_replicates=4, max_cells=3, init={1: 3}, flags=H)
    c["no_hash"] = abi.RunSpec(seed=42, n_replicates=16, max_cells=500, flags=0)
    # snapshots (src/process.rs:122-145): the reference's default 11 cell counts (clap_app.rs:121-134),
    # the pop-front-on-any-match quirk (initial 50 cells, snapshots 1 and 40 popped with 51), and
    # non-monotone birth-death totals
    S = H | abi.FLAG_SNAPSHOT_ROWS
    c["pb_snapshots_default"] = abi.RunSpec(seed=42, n_replicates=16, max_cells=1000,
                                            snapshots=abi.default_snapshots(1000), flags=S)
    c["pb_snapshots_quirk"] = abi.RunSpec(seed=8, n_replicates=16, max_cells=300, init={1: 50},
                                          snapshots=[1, 40, 51, 60, 200, 300], flags=S)
    c["bd_snapshots"] = abi.RunSpec(seed=29, process=abi.BIRTH_DEATH, rates=((1.0, 1.1, 0.9, 0.9),),
                                    n_replicates=32, max_cells=400, init={2: 30}, snapshots=[20, 25, 31, 45, 90],
                                    flags=S | abi.FLAG_TIME_F32)
    c["bd_snapshots_meta_only"] = abi.RunSpec(seed=30, process=abi.BIRTH_DEATH, rates=BD_RATES, n_replicates=32,
                                              max_cells=600, snapshots=abi.default_snapshots(600), flags=H)
    return c


def bin_cases():
    B = abi.FLAG_BIN_STORE
    c = {}
    for name, spec in cases().items():
        c[f"bins_{name}"] = dataclasses.replace(spec, flags=spec.flags | B, _keep=[])
    for name in ("bd_turnover", "big_copies", "abc_sets", "bd_snapshots", "pb_binomial_c1"):
        spec = cases()[name]
        c[f"bins256_{name}"] = dataclasses.replace(spec, flags=spec.flags | B, bin_kmax=256, _keep=[])
    for name in ("bd_binomial", "bd_selection", "spares_mid_copies", "bd_snapshots", "abc_sets", "big_copies"):
        spec = cases()[name]
        c[f"bins32_{name}"] = dataclasses.replace(spec, flags=spec.flags | B, bin_kmax=32, _keep=[])
    c["bins_boundary_pb"] = abi.RunSpec(seed=41, n_replicates=32, max_cells=400, init={30: 2, 33: 1, 64: 2, 65: 2, 130: 1},
                                        hist_bins=300, flags=H | B)
    c["bins_boundary_bd"] = abi.RunSpec(seed=43, process=abi.BIRTH_DEATH, rates=((1.0, 1.3, 0.6, 0.7),),
                                        n_replicates=32, max_cells=500, init={63: 3, 66: 4, 200: 2}, hist_bins=300,
                                        flags=H | B)
    c["bins_boundary_nonminus"] = abi.RunSpec(seed=44, segregation=abi.SEG_BINOMIAL_NO_NMINUS, n_replicates=32,
                                              max_cells=300, init={1: 3, 40: 2, 70: 1}, hist_bins=300, flags=H | B)
    c["bins256_boundary_bd"] = abi.RunSpec(seed=45, process=abi.BIRTH_DEATH, rates=((1.0, 1.3, 0.6, 0.7),),
                                           n_replicates=32, max_cells=500, init={250: 3, 257: 4, 600: 1},
                                           hist_bins=700, bin_kmax=256, flags=H | B)
    # bounded large-k row (big_cap): device rows of 64 cells while outputs keep cell_cap's stride; 40-copy
    # cells divide into two large daughters until the row is full (ECDNA_REP_ERR_CELL_CAP)
    c["bins_big_cap_error"] = abi.RunSpec(seed=48, process=abi.BIRTH_DEATH, rates=((1.0, 1.3, 0.5, 0.5),),
                                          n_replicates=32, max_cells=400, init={40: 6, 1: 4}, bin_kmax=32, big_cap=10,
                                          hist_bins=300, flags=H | B)
    c["bins_big_cap_snapshots"] = abi.RunSpec(seed=49, process=abi.BIRTH_DEATH, rates=((1.0, 1.2, 0.4, 0.4),),
                                              n_replicates=32, max_cells=300, init={36: 3, 2: 5}, bin_kmax=32,
                                              big_cap=200, hist_bins=300, snapshots=[10, 40, 120],
                                              flags=H | B | abi.FLAG_SNAPSHOT_ROWS)
    # Lemire rejections: with a million N+ cells a pick's low product word falls below n+ with probability
    # ~2.3e-4 and is rejected with ~2.25e-4 (2^32 mod 1e6 = 967,296), about 30 rejections over the run
    c["bins_lemire_reject"] = abi.RunSpec(seed=61, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),),
                                          n_replicates=64, max_cells=1_100_000, max_iter=4000, cell_cap=1_100_000,
                                          init={1: 600_000, 3: 400_000}, bin_kmax=32, flags=H | B)
    c["bins_c32"] = abi.RunSpec(seed=46, process=abi.BIRTH_DEATH, rates=BD_RATES, n_replicates=32, max_cells=1500,
                                cell_cap=70_000, init={1: 2, 70: 1}, flags=H | B)
    c["bins256_c32"] = abi.RunSpec(seed=47, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), n_replicates=16,
                                   max_cells=1300, max_time=3.0, cell_cap=70_000, init={1: 900, 80: 100},
                                   bin_kmax=256, flags=H | B | abi.FLAG_SNAPSHOT_ROWS, snapshots=[950, 1000, 1100])
    return c
