/*
 * ecdna_ssa.h — C ABI of the MI355X many-replicate Gillespie SSA engine for
 * ecDNA birth–death–segregation dynamics.
 *
 * This is the drop-in boundary for the reference's hot path. In
 * fraterenz/ecdna-evo v0.26.0 every replicate is one call of
 *
 *     sosa::simulate(&mut state, &rates, &reactions, &mut process, &options, &mut rng)
 *
 * (src/main.rs:92-99 for PureBirth, src/main.rs:166-173 for BirthDeath), made
 * once per replicate index idx by the closure run_simulations
 * (src/main.rs:55-211) that rayon maps over seed*10 .. seed*10+runs
 * (src/main.rs:212-225). Inside that call run the process model
 * (AdvanceStep::advance_step / update_state, src/process.rs:114-197 and
 * src/process.rs:259-345), the event kernels (Exponential::increase_nplus,
 * increase_nminus, CellDeath::decrease_nplus / decrease_nminus,
 * src/proliferation.rs:24-140) and the segregation rules
 * (src/segregation.rs:110-194).
 *
 * Here ONE call runs ALL replicates of a run on one GPU (one replicate per
 * GPU lane): ecdna_ssa_run() replaces the R calls of simulate() that the
 * rayon loop makes, and returns what run_simulations keeps of each one
 * (stop reason, final [n-, n+] and time: src/main.rs:124-128, 198-210) plus
 * the pooled copy-number histogram that process::save writes per replicate
 * (src/process.rs:31-55; JSON body {"0": n-, "k": cells}, dynamics.md:8).
 *
 * Conventions: plain C types only; no exceptions cross the boundary; every
 * buffer is caller-owned; functions return 0 on success or a negative
 * ECDNA_E_* code (ecdna_ssa_strerror). Per-replicate failures that the
 * reference turns into panics are reported in ecdna_rep_summary_t.error.
 *
 * RNG: replicate r (a GLOBAL id, so shards on different GPUs draw the same
 * streams as one big run) uses Philox4x32-10 with key = (seed lo, seed hi)
 * and counter = (event index, sub-block, r lo, r hi). The draw mapping is
 * spelled out in DESIGN.md §3; oracle/ restates it on the CPU bit for bit.
 */
#ifndef ECDNA_SSA_H
#define ECDNA_SSA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI v12: draw mapping v8, the time step as the soft log times the correctly rounded reciprocal RN32(1 / a0) (v7
 * divided: the correctly rounded quotient; the two differ by at most one ulp, so results differ from v11's for the
 * same seed). The Params layout and everything else are those of v11.
 * ABI v11: ECDNA_REP_ERR_INTERNAL (a replicate whose event would pick from an empty N+ set stops instead of
 * indexing off its row); unknown flag bits are rejected; the lane-quad schedule (instance schedule 4) is gone.
 * The Params layout is that of v10 (v10 appended ecdna_ssa_params_t.max_workgroups, a cap on the persistent grid for
 * contexts that share a GPU; v9 took the channel from all 32 bits of the event's word over f64 cumulative
 * propensities, draw mapping v7). */
#define ECDNA_SSA_ABI_VERSION 12

/* Process type — ProcessType (src/clap_app.rs:311-315); chosen as BirthDeath
 * when d0 > 0 or d1 > 0 (src/clap_app.rs:163-174, 194-200). */
typedef enum {
    ECDNA_PURE_BIRTH = 0,  /* channels [ProliferateNMinus, ProliferateNPlus]  src/main.rs:67-71 */
    ECDNA_BIRTH_DEATH = 1  /* + [DeathNMinus, DeathNPlus]                     src/main.rs:139-145 */
} ecdna_process_t;

/* Segregation rule — SegregationOptions (src/clap_app.rs:232-238). */
typedef enum {
    ECDNA_SEG_DETERMINISTIC = 0,      /* Deterministic      src/segregation.rs:142-155 */
    ECDNA_SEG_BINOMIAL = 1,           /* Binomial           src/segregation.rs:110-140 */
    ECDNA_SEG_BINOMIAL_NO_UNEVEN = 2, /* BinomialNoUneven   src/segregation.rs:157-174 */
    ECDNA_SEG_BINOMIAL_NO_NMINUS = 3  /* BinomialNoNminus   src/segregation.rs:176-194 */
} ecdna_seg_t;

/* Reaction channels, in the reference's channel order (src/main.rs:140-145).
 * EcDNAEvent (src/process.rs:20-29) declares 7 variants; only these 4 are
 * reachable (src/process.rs:179, 331). */
typedef enum {
    ECDNA_EV_PROLIF_NMINUS = 0,
    ECDNA_EV_PROLIF_NPLUS = 1,
    ECDNA_EV_DEATH_NMINUS = 2,
    ECDNA_EV_DEATH_NPLUS = 3
} ecdna_event_t;

/* Why a replicate stopped (sosa::StopReason; checked in this order before
 * every event). */
typedef enum {
    ECDNA_STOP_NONE = 0,       /* never started (see error) */
    ECDNA_STOP_MAX_CELLS = 1,  /* n- + n+ >= max_cells        (Options.max_cells, src/clap_app.rs:207) */
    ECDNA_STOP_MAX_TIME = 2,   /* t >= max_time               (IterTime.time, src/clap_app.rs:205) */
    ECDNA_STOP_MAX_ITER = 3,   /* iterations >= max_iter      (MAX_ITER, src/main.rs:23) */
    ECDNA_STOP_ABSORBING = 4,  /* total propensity == 0 (extinction) */
    ECDNA_STOP_ERROR = 5       /* see ecdna_rep_summary_t.error */
} ecdna_stop_t;

/* Per-replicate errors — where the reference panics or refuses. */
typedef enum {
    ECDNA_REP_OK = 0,
    ECDNA_REP_ERR_OVERFLOW = 1,   /* 2k > u16::MAX: checked_mul panic, src/proliferation.rs:63-67 */
    ECDNA_REP_ERR_EMPTY = 2,      /* empty initial distribution: ensure!, src/process.rs:88, 232 */
    ECDNA_REP_ERR_CELL_CAP = 3,   /* N+ row would exceed cell_cap (the reference grows a Vec), or the
                                     bin store's large-k row would exceed big_cap */
    ECDNA_REP_ERR_REJECTION = 4,  /* BinomialNoUneven loop exceeded 4096 redraws (p < 2^-4096) */
    ECDNA_REP_ERR_INTERNAL = 5    /* an N+ event drawn with no N+ cell, or a cell index past n+ (ABI v11): the event
                                     is not applied and the replicate stops. Unreachable under draw mapping v8 (a
                                     zero-propensity channel is never drawn); the guard keeps a broken invariant
                                     from indexing off the row. The reference's pick_remove_random_nplus returns an
                                     error on an empty N+ set (src/proliferation.rs:57). */
} ecdna_rep_error_t;

/* Flags (ecdna_ssa_params_t.flags). */
#define ECDNA_FLAG_TIME_F32 0x1u       /* accumulate time in f32 like process.time (src/process.rs:68, 184) */
#define ECDNA_FLAG_BD_CAP_COMPAT 0x2u  /* BD: stop at 2(n- + n+) >= max_cells, i.e. sum of the
                                          duplicated population vector (src/process.rs:339-344) */
#define ECDNA_FLAG_EVENT_HASH 0x4u     /* fold every event into ecdna_rep_summary_t.event_hash */
#define ECDNA_FLAG_SNAPSHOT_ROWS 0x8u  /* keep the N+ row of every snapshot (else only its metadata) */
#define ECDNA_FLAG_REP_STATS 0x10u     /* per-replicate ABC statistics (ecdna_rep_stats_t) */
/* Cell store of a replicate's N+ cells. Default: the ROW store, one u16 per cell
 * in the reference's swap_remove order (ecdna-lib EcDNADistribution.nplus: Vec<u16>). With this flag:
 * the BIN store, per-replicate counts of cells by copy number k = 1..bin_kmax held in LDS, plus a
 * row of the cells with k > bin_kmax. A uniform cell pick has the same law under any arrangement
 * of the cells, so both stores simulate the same process; they consume the same draws but address
 * cells in a different order, so their runs differ seed for seed (each is bit-exact with its own
 * oracle restatement). Final and snapshot rows come back in canonical order: k = 1 cells, k = 2
 * cells, ..., k = bin_kmax cells, then the large-k row. */
#define ECDNA_FLAG_BIN_STORE 0x20u
/* Reference draw structure (row store only; not with ECDNA_FLAG_BIN_STORE): instead of the engine's Philox
 * mapping, replicate r draws exactly what the Rust reference draws for replicate index r — ChaCha8Rng
 * seed_from_u64(seed) on stream seed*10 + r (src/main.rs:56-58), the first-reaction method over f32
 * propensities with rand_distr's Exp1 ziggurat, gen_range + swap_remove for cell picks, rand_distr's
 * Binomial (BINV / BTPE) for segregation — and accumulates time in f32 (process.time, src/process.rs:184;
 * ECDNA_FLAG_TIME_F32 is implied). log and exp are the correctly rounded functions (the reference's glibc
 * calls agree with them wherever glibc rounds correctly). A correctness path for seed-for-seed comparison
 * with the reference semantics, not a fast path. */
#define ECDNA_FLAG_REFERENCE_DRAWS 0x40u
/* Every defined flag; ecdna_ssa_ctx_create rejects other bits (ABI v11). */
#define ECDNA_FLAG_ALL 0x7fu

/* API return codes. */
#define ECDNA_OK 0
#define ECDNA_E_INVALID (-1)   /* bad parameter */
#define ECDNA_E_HIP (-2)       /* HIP runtime error */
#define ECDNA_E_NOMEM (-3)     /* device allocation failed */
#define ECDNA_E_NODEVICE (-4)  /* no usable gfx950 device */
#define ECDNA_E_STATE (-5)     /* call order (e.g. download before launch) */
#define ECDNA_E_COMM (-6)      /* RCCL error, or librccl.so.1 not loadable (multi-GPU reduction only) */

/* Rates of one parameter set: ReactionRates([b0, b1, d0, d1]) (src/main.rs:67, 139). f32 as in Cli
 * (src/clap_app.rs:41-55). Each must be 0 or in [2^-60, 2^60] (else ECDNA_E_INVALID; the reference does not
 * check them; since ABI v8): the f32 propensities (rate x population, u32 populations) and the f32 total a0 of
 * the time step then stay normal and finite, which the stepper's time-step division relies on. */
typedef struct {
    float b0, b1, d0, d1;
} ecdna_rates_t;

/* One run = n_replicates independent replicates; replicate i of the call (i = 0 .. n_replicates - 1)
 * has global id r = first_replicate + i * replicate_stride (stride 0 or 1: the contiguous ids
 * first_replicate .. first_replicate + n_replicates - 1). Replicate r uses parameter set
 * s = r / reps_per_set (must be < n_param_sets). Every draw is keyed by r, so a replicate's results do
 * not depend on which call, device or position runs it: G calls with first_replicate = g and
 * replicate_stride = G (g = 0 .. G-1) together run the same replicates as one call, interleaved so
 * that every call gets the same mix of parameter sets (balanced ABC sweeps across GPUs). */
typedef struct {
    int32_t process;                /* ecdna_process_t */
    int32_t segregation;            /* ecdna_seg_t */
    const ecdna_rates_t* rates;     /* host, [n_param_sets] */
    uint32_t n_param_sets;          /* 1, or e.g. 1024 for an ABC sweep */
    uint32_t hist_bins;             /* bins per set: bin 0 = N- cells, bin k = cells with k copies,
                                       bin hist_bins-1 = cells with >= hist_bins-1 copies; >= 2 */
    uint64_t reps_per_set;          /* replicates per parameter set (>= 1) */
    uint64_t seed;                  /* --seed (src/clap_app.rs:63) */
    uint64_t first_replicate;       /* global id of the first replicate of this call (sharding) */
    uint64_t n_replicates;          /* replicates in this call */
    uint64_t max_cells;             /* stop when n- + n+ >= max_cells (src/clap_app.rs:142-157) */
    double max_time;                /* stop when t >= max_time (years; src/clap_app.rs:151, 205) */
    uint64_t max_iter;              /* stop after max_iter events (1e9, src/main.rs:23); < 2^32 */
    uint32_t cell_cap;              /* capacity of the per-replicate N+ row (cells); rounded up to 64 */
    uint32_t flags;                 /* ECDNA_FLAG_* */
    /* Initial distribution (EcDNADistribution: n- plus one u16 per N+ cell; default {1: 1},
     * src/clap_app.rs:188-191). Either shared by every set (init_set_offsets == NULL: copies
     * init_copies[0 .. init_nplus), n- = init_nminus) or per set (init_set_offsets[n_param_sets+1]
     * into init_copies, init_set_nminus[n_param_sets]). Copy numbers must be >= 1. */
    const uint16_t* init_copies;    /* host */
    uint32_t init_nplus;
    uint32_t bin_kmax;              /* ECDNA_FLAG_BIN_STORE: copy numbers 1..bin_kmax are binned; 32, 64 or
                                       256 (0 = 64); part of the draw mapping (the canonical cell order) */
    uint64_t init_nminus;
    const uint32_t* init_set_offsets; /* host or NULL */
    const uint64_t* init_set_nminus;  /* host or NULL */
    int32_t device;                 /* HIP device ordinal for ecdna_ssa_run / ctx_create */
    uint32_t big_cap;               /* ECDNA_FLAG_BIN_STORE: capacity (cells) of a replicate's large-k row,
                                       the cells with k > bin_kmax; 0 = cell_cap. A division that would put
                                       more cells there stops the replicate with ECDNA_REP_ERR_CELL_CAP. The
                                       device row memory is sized by it, outputs by cell_cap. */
    /* Snapshots (--snapshots, src/clap_app.rs:92-97, 102-134; SavingOptions, src/lib.rs:21-25): cell
     * counts, sorted ascending, at most 64. Before every event, while any REMAINING snapshot equals
     * n- + n+, the FRONT one is popped and the current state saved (src/process.rs:122-145, the
     * reference's pop_front-on-any-match rule). NULL / 0 = none. */
    const uint64_t* snapshot_cells; /* host */
    uint32_t n_snapshots;
    uint32_t replicate_stride;      /* global-id step between consecutive replicates of the call (0 = 1) */
    /* Per-replicate ABC summary statistics (abc.md:38-55; ECDNA_FLAG_REP_STATS): compared against this
     * target copy-number histogram of hist_bins entries (bin 0 = N- cells, last bin = overflow), e.g.
     * the patient's data. NULL: statistics are computed, distances to the target are not. */
    const uint64_t* stats_target_hist; /* host */
    /* Scheduling hint (optional, host, n_param_sets entries): the relative cost of one replicate of each
     * parameter set. Replicates of costlier sets are started first (longest-processing-time order, ties
     * in id order), which shortens the tail of a run whose sets differ in cost, such as an ABC sweep.
     * Results do not depend on it. NULL: replicates start in id order. */
    const float* set_cost_hint;
    /* Persistent-grid cap (since ABI v10): at most this many workgroups (0 = as many as the kernel's occupancy
     * fits on the device). Two contexts launched on two streams of one GPU share its CUs only when their grids
     * leave room for each other, e.g. a shard split by initial copy number onto two bin-store instances
     * (DESIGN.md §7). Results do not depend on it. */
    uint32_t max_workgroups;
    uint32_t reserved0;             /* must be 0 */
} ecdna_ssa_params_t;

/* Per-replicate summary statistics of the final distribution (cells = n- + n+, copy number k per cell,
 * k = 0 for N- cells; bins as in the histogram). Distances are against params.stats_target_hist. */
typedef struct {
    double mean;           /* sum k / cells                                           */
    double entropy;        /* -sum_k p_k ln p_k, p_k = cells with k copies / cells     */
    double frequency;      /* n+ / cells                                              */
    double ks;             /* max_k |F(k) - F_target(k)|, F = cumulative p over bins  */
    double mean_rel;       /* |mean - mean_t| / mean_t      (|mean - mean_t| if mean_t == 0) */
    double entropy_rel;    /* |entropy - entropy_t| / entropy_t (likewise)            */
    double frequency_diff; /* |frequency - frequency_t|                               */
    uint64_t cells;
} ecdna_rep_stats_t;

/* One saved snapshot of one replicate (what process::save writes, src/process.rs:31-55). */
typedef struct {
    double time;                    /* process.time at the save (before the event's waiting time) */
    uint64_t nminus;
    uint64_t nplus;
    uint32_t taken;                 /* 1 if this snapshot was popped (saved) during the run */
    uint32_t reserved;
} ecdna_snapshot_t;

/* What run_simulations keeps of one replicate (src/main.rs:124-128, 198-210), plus counters. */
typedef struct {
    uint64_t nminus;                /* final n-  (population[0]) */
    uint64_t nplus;                 /* final n+  (population[1]) */
    uint64_t iters;                 /* events executed = advance_step calls */
    uint64_t events_by_type[4];     /* per ecdna_event_t */
    uint64_t uneven;                /* ProliferateNPlus events with a complete uneven split */
    double time;                    /* final process.time (years) */
    uint64_t event_hash;            /* FNV-1a fold of (event, k1, cell index) per event, if enabled */
    uint32_t stop_reason;           /* ecdna_stop_t */
    uint32_t error;                 /* ecdna_rep_error_t */
} ecdna_rep_summary_t;

/* Per-parameter-set sums over the replicates of a call. */
typedef struct {
    uint64_t replicates;
    uint64_t events;                /* sum of iters — the numerator of events/s */
    uint64_t events_by_type[4];
    uint64_t uneven;
    uint64_t nminus;                /* sum of final n- */
    uint64_t nplus;                 /* sum of final n+ */
    uint64_t stop_reasons[6];       /* per ecdna_stop_t */
    uint64_t errors;                /* replicates with error != 0 */
} ecdna_totals_t;

int ecdna_ssa_abi_version(void);
const char* ecdna_ssa_strerror(int code);
/* Detail of the last failure on the calling thread ("" if none). */
const char* ecdna_ssa_last_error_message(void);

/* Number of usable gfx950 devices (0 when none). */
int ecdna_ssa_device_count(void);

/* One-shot: runs every replicate of *p on device p->device and copies the results to HOST buffers
 * (each may be NULL): out_summaries[n_replicates] (replicate first_replicate + i * stride at index i),
 * out_hist[n_param_sets * hist_bins] (zeroed, then filled), out_totals[n_param_sets].
 * stream: a hipStream_t, or NULL for the default (null) stream. Blocks until done. */
int ecdna_ssa_run(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries,
                  uint64_t* out_hist, ecdna_totals_t* out_totals, void* stream);

/* Device-resident context for repeated runs (benchmarks, multi-GPU). Inputs are uploaded once at
 * create; rows/summaries/histogram stay in HBM between launches. */
typedef struct ecdna_ssa_ctx ecdna_ssa_ctx;

int ecdna_ssa_ctx_create(const ecdna_ssa_params_t* p, ecdna_ssa_ctx** out);
/* Use caller-owned DEVICE buffers for the histogram [n_param_sets*hist_bins] u64 and totals
 * [n_param_sets] (e.g. tensors later all-reduced over RCCL). NULL keeps the internal buffer. */
int ecdna_ssa_ctx_set_outputs(ecdna_ssa_ctx* c, uint64_t* d_hist, ecdna_totals_t* d_totals);
/* Enqueue one full run on `stream` (a hipStream_t; NULL = the default stream): zero hist/totals, SSA
 * kernel over all replicates (in memory-bounded chunks), histogram kernel. Asynchronous. */
int ecdna_ssa_ctx_launch(ecdna_ssa_ctx* c, void* stream);
/* Block until the last launch finished; returns its device time in ms (HIP events on the launch
 * stream): ssa_ms = SSA stepper kernels only, hist_ms = histogram/summary kernels. Either may be NULL. */
int ecdna_ssa_ctx_sync(ecdna_ssa_ctx* c, float* ssa_ms, float* hist_ms);
/* Device pointers of the current outputs. */
int ecdna_ssa_ctx_device_outputs(ecdna_ssa_ctx* c, uint64_t** d_hist, ecdna_totals_t** d_totals);
/* Copy results of the last launch to HOST buffers (each may be NULL). out_rows, if given, receives
 * [n_replicates][row_stride] u16 where row i holds the final N+ copies of replicate i in the
 * engine's swap_remove order (row store) or in canonical order (bin store, ECDNA_FLAG_BIN_STORE);
 * entries past summaries[i].nplus are unspecified. Valid only when the
 * whole run fit in one chunk (ecdna_ssa_ctx_row_stride returns > 0). */
int ecdna_ssa_ctx_download(ecdna_ssa_ctx* c, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                           ecdna_totals_t* out_totals, uint16_t* out_rows);
/* Snapshots of the last launch: meta[n_replicates][n_snapshots] and, under ECDNA_FLAG_SNAPSHOT_ROWS,
 * rows[n_replicates][n_snapshots][row_stride] u16 (the N+ cells at the save, in the order of
 * ecdna_ssa_ctx_download).
 * Either may be NULL. */
int ecdna_ssa_ctx_download_snapshots(ecdna_ssa_ctx* c, ecdna_snapshot_t* meta, uint16_t* rows);
/* Per-replicate statistics of the last launch (needs ECDNA_FLAG_REP_STATS): out[n_replicates]. */
int ecdna_ssa_ctx_download_stats(ecdna_ssa_ctx* c, ecdna_rep_stats_t* out);
/* Reference draws (ECDNA_FLAG_REFERENCE_DRAWS, ABI v7): per replicate, the number of 32-bit words its ChaCha8
 * stream (seed_from_u64(seed), stream seed*10 + r) had handed out when it stopped — where the reference's
 * end-of-run subsampling continues the same rng (into_subsampled(nb, &mut rng), src/main.rs:110-123, 184-197;
 * ecdna_host_subsample_reference). out[n_replicates]. */
int ecdna_ssa_ctx_download_rng_words(ecdna_ssa_ctx* c, uint64_t* out);
/* Row stride (cells) of the rows buffer, or 0 when the run is chunked (rows not downloadable). */
int64_t ecdna_ssa_ctx_row_stride(const ecdna_ssa_ctx* c);
/* Replicates per chunk (memory bound) and lanes of the persistent stepper grid. */
int ecdna_ssa_ctx_geometry(const ecdna_ssa_ctx* c, uint64_t* chunk_replicates, uint64_t* grid_lanes);

/* The kernel instance a context launches (ABI v7): every choice ecdna_ssa_ctx_create makes from the
 * workload shape and the ECDNA_SSA_* environment knobs, so that a benchmark line can name
 * the instance it timed and a flip of an automatic rule shows up in its output. Results never depend on
 * any of these; they are speed choices. */
typedef enum {
    ECDNA_KERNEL_ROWS = 0,       /* ssa_stepper: the row store (one u16 per cell in HBM) */
    ECDNA_KERNEL_BINS = 1,       /* ssa_stepper_bins: the bin store (ECDNA_FLAG_BIN_STORE) */
    ECDNA_KERNEL_REFDRAWS = 2    /* ssa_stepper_refdraws: the reference draws (ECDNA_FLAG_REFERENCE_DRAWS) */
} ecdna_kernel_kind_t;
typedef struct {
    int32_t kernel;            /* ecdna_kernel_kind_t */
    int32_t schedule;          /* bin stepper: 0 occupancy-first, 1 max-ILP, 2 occupancy-first capped at 128
                                  VGPRs (K = 64 / u16), 3 max-ILP with paired lanes; -1 for the other kernels */
    int32_t paired;            /* 1: lane l < 32 owns a replicate, lane l + 32 helps its N- fast-forward (pairs) */
    int32_t rotation;          /* number of chunks whose replicates rotate through the lanes */
    int32_t rot_tick_log2;     /* rotation tick (loop iterations, log2) */
    int32_t drain_control;     /* number of chunks whose youngest wave slots stop admitting replicates early */
    int32_t cost_order;        /* 1: replicates start costliest set first (params.set_cost_hint) */
    int32_t runtime_flags;     /* 1: the instance reads f32 time, the event hash and snapshots from its arguments
                                  (TF = 1); 0: compiled out */
    uint32_t bin_kmax;         /* bin store: binned copy numbers (0 for the other kernels) */
    uint32_t bin_c32;          /* bin store: 1 = u32 counters, 0 = u16 */
    uint32_t block_lanes;      /* workgroup size */
    uint32_t blocks_per_cu;    /* workgroups per CU of the launched grid (rounded up; largest chunk) */
    uint32_t cus;              /* compute units of the device */
    uint32_t n_chunks;         /* launches per run (HBM-bounded chunks) */
    uint32_t vgprs;            /* per lane, as compiled (hipFuncGetAttributes numRegs) */
    uint32_t lds_bytes;        /* static LDS per workgroup */
    uint32_t scratch_bytes;    /* private segment per lane */
    uint32_t window;           /* row store: 1 = LDS tail window variant */
    uint64_t chunk_replicates; /* replicates per chunk */
    uint64_t grid_lanes;       /* lanes of the launched grid (largest chunk; <= the occupancy cap) */
} ecdna_ssa_instance_t;
int ecdna_ssa_ctx_instance(const ecdna_ssa_ctx* c, ecdna_ssa_instance_t* out);
int ecdna_ssa_ctx_destroy(ecdna_ssa_ctx* c);

/* ---- Multi-GPU reduction (ABI v6; RCCL over xGMI).
 * Replicates shard over GPUs by GLOBAL id (first_replicate / replicate_stride), so every shard draws exactly
 * the streams the same replicates draw in one big run, and the whole run's histogram and totals are the
 * element-wise sum of the shards' — one all-reduce (ncclUint64, ncclSum), exact and order-independent. This
 * replaces the reference's collection of per-replicate results from its rayon loop (src/main.rs:221-224)
 * when the replicates live on several GPUs.
 * A communicator is an RCCL ncclComm_t passed as void*: made here (ecdna_ssa_comm_init_all for one process
 * driving several devices, one host thread per device; ecdna_ssa_comm_init_rank for one process per device
 * with the unique id of ecdna_ssa_comm_unique_id shared by the caller), or made by the caller with RCCL. RCCL
 * (librccl.so.1) is loaded at the first of these calls; without it they return ECDNA_E_COMM. */
#define ECDNA_COMM_ID_BYTES 128
int ecdna_ssa_comm_unique_id(uint8_t out_id[ECDNA_COMM_ID_BYTES]);
int ecdna_ssa_comm_init_rank(const uint8_t id[ECDNA_COMM_ID_BYTES], int n_ranks, int rank, int device,
                             void** out_comm);
/* out_comms[n_devices]: one communicator per device of devices[] (ncclCommInitAll). */
int ecdna_ssa_comm_init_all(int n_devices, const int* devices, void** out_comms);
int ecdna_ssa_comm_destroy(void* comm);
/* In-place all-reduce (sum) over `comm` of a run's DEVICE histogram [n_param_sets * hist_bins] u64 and totals
 * [n_param_sets], enqueued on `stream` (a hipStream_t; NULL = default). Every rank of the communicator must
 * call it with the same n_param_sets and hist_bins. Asynchronous. */
int ecdna_ssa_reduce_hist(void* comm, uint64_t* d_hist, ecdna_totals_t* d_totals, uint32_t n_param_sets,
                          uint32_t hist_bins, void* stream);
/* The same on a context's current outputs (ecdna_ssa_ctx_set_outputs or its own), on the stream of its last
 * launch; ecdna_ssa_ctx_download then returns the reduced histogram and totals. */
int ecdna_ssa_ctx_reduce(ecdna_ssa_ctx* c, void* comm);

#ifdef __cplusplus
}
#endif

#endif /* ECDNA_SSA_H */
