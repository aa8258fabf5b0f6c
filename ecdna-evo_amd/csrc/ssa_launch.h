// ssa_launch.h — host-visible kernel argument blocks and launch wrappers shared by
// ssa_kernels.hip (device code) and ssa_api.cpp (the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ecdna_ssa.h"

namespace ecdna {

// Replicate rotation (bin store): replicates are split into kRotParts partitions, one per XCD (the
// XCC id of the lane's CU), so a parked replicate is only ever resumed by a CU that shares the L2 it
// was parked through. Partition x holds the replicates r with r mod kRotParts == x; its waiting
// replicates are found by walking its items: item j is replicate x + kRotParts * (j % rot_n_pad) (pass
// j / rot_n_pad: round-robin order; slots past the chunk are DONE); rot_n_pad is a multiple of kRotBlock.
constexpr uint32_t kRotParts = 8;
constexpr uint32_t kRotBlock = 16;
constexpr uint32_t kParkVecs = 4;    // 64 B of scalars per parked replicate
enum RotState : uint32_t { ROT_FRESH = 0, ROT_RUNNING = 1, ROT_PARKED = 2, ROT_DONE = 3 };
struct alignas(128) RotPart {
    unsigned long long head;        // items walked
    int waiting;                    // FRESH + PARKED replicates (never below the number of such flags)
    int fresh;                      // FRESH replicates
    uint32_t pad[28];
};

// One chunk of replicates for the persistent SSA stepper.
struct StepperArgs {
    uint16_t* rows;                 // [n][row_stride] per-replicate N+ rows (replicate-major)
    ecdna_rep_summary_t* summaries; // [n], already offset to the chunk
    uint32_t* head;                 // work counter (zeroed before the launch)
    const uint32_t* order;          // [n] chunk-local start order (costliest sets first) or nullptr: id order
    const float4* rates;            // [n_param_sets] (b0, b1, d0, d1)
    const uint16_t* init_copies;
    const uint32_t* init_offsets;   // [n_sets + 1] or nullptr (shared initial distribution)
    const uint64_t* init_nminus_set;// [n_sets] or nullptr
    uint64_t row_stride;            // cells per row (multiple of 64 -> 128-B aligned rows)
    uint64_t seed;
    uint64_t rid0;                  // global id of the chunk's first replicate
    uint64_t rid_stride;            // global-id step between the chunk's replicates (>= 1)
    uint64_t reps_per_set;
    uint64_t max_cells;
    uint64_t stop_cells;            // MaxCells when n- + n+ >= stop_cells: max_cells, or
                                    // ceil(max_cells / 2) under ECDNA_FLAG_BD_CAP_COMPAT (birth-death)
    uint64_t init_nminus;
    double max_time;
    float max_time32;
    uint32_t n;                     // replicates in the chunk
    uint32_t init_nplus;
    uint32_t max_iter;
    uint32_t cell_cap;
    uint32_t flags;
    uint32_t n_snap;                // snapshots (0 = none)
    const uint64_t* snap_cells;     // [n_snap], ascending
    ecdna_snapshot_t* snap_meta;    // [n][n_snap], chunk-offset
    uint16_t* snap_rows;            // [n][n_snap][snap_stride] or nullptr, chunk-offset
    uint64_t snap_stride;           // cells per snapshot row (cell_cap rounded up)
    uint32_t big_cap;               // bin store: large-k row capacity (<= cell_cap, <= row_stride)
    void* bags;                     // bin store: [n][bin_k] final u16 / u32 bin counters (chunk-local)
    // bin store drain control: waves in SIMD wave slots >= admit_slot (the youngest) take no fresh
    // replicate once fewer than admit_remaining are left; admit_slot = 0xffffffff: off
    uint32_t admit_slot;
    uint32_t admit_remaining;
    // bin store replicate rotation ("Rotation"): every 2^rot_tick_log2 loop iterations a
    // wave parks its lanes' replicates (bin counters -> bags, scalars -> park) and its lanes pull the next
    // waiting replicate of their XCD's partition, so all replicates advance together and none starts
    // late. rot_parts = nullptr: off.
    RotPart* rot_parts;             // [kRotParts] (host-initialised per launch)
    uint32_t* rot_flags;            // [kRotParts * rot_n_pad]: RotState per replicate
    uint4* rot_park;                // [n][kParkVecs] parked scalars
    uint32_t rot_n_pad;             // replicates per partition, multiple of kRotBlock
    uint32_t rot_tick_log2;
    int32_t rot_park_min;           // park at a tick only if at least this many replicates wait
    // reference draws (ECDNA_FLAG_REFERENCE_DRAWS, ssa_refdraws.hip): the ChaCha8 key of seed_from_u64(seed)
    // (8 words) and the BTPE constants of Binomial(2k, 1/2) per copy number k (refdraws::kBtpeRow doubles)
    const uint32_t* ref_key;
    const double* ref_btpe;
    uint64_t* rng_words;            // [n] chunk-offset: ChaCha8 words each replicate's stream handed out (or nullptr)
};

// Histogram / totals pass over one chunk.
struct HistArgs {
    const uint16_t* rows;
    const ecdna_rep_summary_t* summaries; // chunk-offset
    uint64_t* hist;                       // [n_sets][bins]
    unsigned long long* totals;           // [n_sets][16] (ecdna_totals_t as u64 words)
    uint64_t row_stride;
    uint64_t rid0;
    uint64_t rid_stride;                  // >= 1
    uint64_t reps_per_set;
    uint32_t n;
    uint32_t bins;
    uint32_t reps_per_block;
    // per-replicate ABC statistics (nullptr = off), against target_cdf[bins] when has_target
    ecdna_rep_stats_t* stats;             // chunk-offset
    const double* target_cdf;
    double target_mean, target_entropy, target_freq;
    uint32_t has_target;
    // bin store: per-replicate counters [n][bag_k] (u16, or u32 when bag_c32); nullptr = rows only
    const void* bags;
    uint32_t bag_k;
    uint32_t bag_c32;
};

constexpr int kStepperBlock = 256;
constexpr int kBinWideBlock = 64;  // bin store with 256 bins
constexpr int kHistBlock = 256;
constexpr uint32_t kMaxHistBins = 4096;  // LDS: 8 B per bin per workgroup (<= 64 KiB)
constexpr uint32_t kMaxSnapshots = 64;
// Internal flag bit (never a user flag): the run takes snapshots. With f32 time and the event hash it selects the bin
// stepper's runtime-flags instances (TF = 1); the TF = 0 instances (the bench's) compile snapshots, f32 time and the
// hash out, which frees the scalar registers the snapshot test held across the event loop.
constexpr uint32_t kFlagSnapshotsRt = 0x80000000u;
constexpr uint32_t kRuntimeFlagMask = ECDNA_FLAG_TIME_F32 | ECDNA_FLAG_EVENT_HASH | kFlagSnapshotsRt;

// Kernel handle for occupancy queries and the launch itself.
// window: 1 = LDS tail window variant (default), 0 = rows straight in HBM (A/B reference)
const void* stepper_kernel(int birth_death, int segregation, int window);
hipError_t launch_stepper(const StepperArgs& a, int birth_death, int segregation, int window, uint32_t blocks,
                          hipStream_t stream);
// Bin store (ECDNA_FLAG_BIN_STORE): bin_k = 64 or 256 binned copy numbers; c32 = u32 counters
// (cell_cap > 65535); flags selects the compile-time variant without f32 time and event hash when
// neither is set. bin_stepper_block = the variant's workgroup size.
// ilp: 1 = the max-ILP instruction schedule of the same kernels (a second compile of ssa_kernels.hip,
// ECDNA_ILP_BUILD): fewer stalls for lone waves, more VGPRs (3 waves per SIMD); the ABI takes it when a
// chunk has at most one wave of replicates per SIMD. ilp = 2: for K = 64 / u16, the
// default schedule capped at 128 VGPRs (4 workgroups per CU instead of 3), taken when lanes run many
// replicates each; other K / counter widths fall back to the default schedule.
const void* bin_stepper_kernel(int birth_death, int segregation, uint32_t bin_k, int c32, uint32_t flags, int ilp);
const void* bin_stepper_kernel_ilp(int birth_death, int segregation, uint32_t bin_k, int c32, uint32_t flags);
// ilp = 3: the max-ILP schedule with paired lanes (lane l < 32 owns a replicate, lane l + 32 helps its N-
// fast-forward; birth-death, K = 32 / u32 or K = 64): nullptr where no such instance exists. A paired
// workgroup of kStepperBlock lanes runs kStepperBlock / 2 replicates at a time.
const void* bin_stepper_kernel_pair(int segregation, uint32_t bin_k, int c32, uint32_t flags);
int bin_stepper_block(uint32_t bin_k);
hipError_t launch_bin_stepper(const StepperArgs& a, int birth_death, int segregation, uint32_t bin_k, int c32, int ilp,
                              uint32_t blocks, hipStream_t stream);
hipError_t launch_hist(const HistArgs& a, uint32_t blocks, hipStream_t stream);
// The reference-draws stepper (row store; ssa_refdraws.hip)
const void* refdraws_kernel(int birth_death, int segregation);
int refdraws_block();
hipError_t launch_refdraws(const StepperArgs& a, int birth_death, int segregation, uint32_t blocks,
                           hipStream_t stream);

}  // namespace ecdna
