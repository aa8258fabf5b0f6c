// dynamics_main.cpp — `ecdna-dynamics`, the native host of the MI355X engine. It mirrors the
// reference binary: the clap CLI (src/clap_app.rs:26-229, same flags, defaults and conflicts) and
// main() (src/main.rs:46-229): every replicate idx in seed*10 .. seed*10+runs is simulated — here all
// of them in one batched call per GPU through the C ABI (include/ecdna_ssa.h) instead of one
// sosa::simulate call per rayon task — and its snapshots, final distribution and subsamples are saved
// as JSON histograms under DIR exactly where process::save puts them (src/process.rs:31-55).
//
// Additions: --gpus N (replicate shards on N devices, one host thread each), --time {f32,f64}
// (default f32 = the reference's process.time), --cell-cap (row capacity; needed with --years),
// --hist-bins, --dry-run (print the resolved options as JSON and exit), --cell-store {bins,rows}
// (default bins: copy-number counters in LDS), --bin-kmax {64,256}, --draws
// {philox,reference} (reference: the Rust binary's own draw structure, ChaCha8 + rand_distr, seed for seed;
// row store) and --pooled FILE (the run's pooled copy-number histogram and totals, all-reduced over the
// GPUs with RCCL through ecdna_ssa_ctx_reduce, written as JSON).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <ctime>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ecdna_ssa.h"
#include "ecdna_host.hpp"

using ecdna::host::Distribution;

namespace {

constexpr uint64_t kMaxIter = 1000000000ull;   // MAX_ITER, src/main.rs:23
constexpr uint64_t kMaxCells = 1000000000ull;  // MAX_CELLS, src/main.rs:25

struct Options {
    int segregation = ECDNA_SEG_BINOMIAL;
    std::string segregation_name = "binomial";
    std::string growth = "exponential";
    float b0 = 1.f, b1 = 1.f;
    std::string b0_arg = "1", b1_arg = "1", d0_arg = "0", d1_arg = "0";  // as given (for error messages)
    bool has_d0 = false, has_d1 = false;
    float d0 = 0.f, d1 = 0.f;
    bool has_years = false, has_cells = false;
    uint64_t years = 0, cells = 0;
    uint64_t seed = 26;
    bool debug = false, sequential = false;
    std::string path;
    std::string initial;
    bool has_runs = false;
    uint64_t runs = 12;
    std::vector<uint64_t> subsamples;
    bool has_snapshots = false;
    std::vector<uint64_t> snapshots;
    int verbosity = 0;
    // additions
    int gpus = 1;
    bool time_f64 = false;
    uint64_t cell_cap = 0;
    uint32_t hist_bins = 1025;
    bool dry_run = false;
    bool rows = false;       // --cell-store rows
    uint32_t bin_kmax = 64;  // --bin-kmax
    bool has_cell_store = false, has_bin_kmax = false;
    bool reference_draws = false;  // --draws reference
    std::string pooled;            // --pooled FILE
};

[[noreturn]] void usage_error(const std::string& msg) {
    std::fprintf(stderr, "error: %s\n\nUsage: ecdna-dynamics [OPTIONS] <DIR>\n", msg.c_str());
    std::exit(2);
}

void print_help() {
    std::printf(
        "Study the effect of the random segregation and positive selection on the ecDNA dynamics using a\n"
        "stochastic simulation algorithm (SSA) aka Gillespie algorithm — MI355X engine\n\n"
        "Usage: ecdna-dynamics [OPTIONS] <DIR>\n\n"
        "Arguments:\n  <DIR>  Path to store the results of the simulations\n\n"
        "Options:\n"
        "      --segregation <SEGREGATION>  [default: binomial] [possible values: deterministic,\n"
        "                                   binomial-no-uneven, binomial, binomial-no-nminus]\n"
        "      --growth <GROWTH>            [default: exponential] [possible values: exponential, constant]\n"
        "      --b0 <RATE>                  Proliferation rate of the cells without ecDNAs [default: 1]\n"
        "      --b1 <RATE>                  Proliferation rate of the cells with ecDNAs [default: 1]\n"
        "      --d0 <RATE>                  Death rate of the cells without ecDNAs\n"
        "      --d1 <RATE>                  Death rate of the cells with ecDNAs\n"
        "  -y, --years <YEARS>              Number of years to simulate\n"
        "  -c, --cells <CELLS>              Number of cells to simulate\n"
        "      --seed <SEED>                [default: 26]\n"
        "  -d, --debug                      1 sequential run of 300 cells, max verbosity\n"
        "  -s, --sequential                 Run sequentially (one GPU)\n"
        "      --initial <FILE>             JSON initial distribution\n"
        "  -r, --runs <RUNS>                [default: 12]\n"
        "      --subsamples=<N,...>         Subsample the ecDNA distribution at the end\n"
        "      --snapshots=<N,...>          Cell counts that trigger saving the distribution\n"
        "  -v, --verbosity...               \n"
        "      --gpus <N>                   GPUs to shard the replicates over [default: 1]\n"
        "      --time <f32|f64>             time accumulation [default: f32]\n"
        "      --cell-cap <CELLS>           N+ row capacity [default: cells, or 2^24 with --years]\n"
        "      --hist-bins <BINS>           [default: 1025]\n"
        "      --dry-run                    print the resolved options as JSON and exit\n"
        "      --cell-store <bins|rows>     N+ cell store of the engine [default: bins]\n"
        "      --bin-kmax <64|256>          copy numbers held as counters by the bin store [default: 64]\n"
        "      --draws <philox|reference>   random draws: the engine's Philox mapping, or the reference's\n"
        "                                   own (ChaCha8 + rand_distr, seed for seed; row store) [default: philox]\n"
        "      --pooled <FILE>              write the run's pooled histogram and totals (RCCL-reduced) as JSON\n"
        "  -h, --help                       Print help\n");
}

uint64_t parse_u64(const std::string& flag, const std::string& v) {
    if (v.empty() || v.find_first_not_of("0123456789") != std::string::npos)
        usage_error("invalid value '" + v + "' for '" + flag + "'");
    return std::strtoull(v.c_str(), nullptr, 10);
}

float parse_f32(const std::string& flag, const std::string& v) {
    char* end = nullptr;
    float x = std::strtof(v.c_str(), &end);
    if (v.empty() || *end) usage_error("invalid value '" + v + "' for '" + flag + "'");
    return x;
}

std::vector<uint64_t> parse_list(const std::string& flag, const std::string& v) {
    std::vector<uint64_t> out;
    size_t i = 0;
    while (i <= v.size() && !v.empty()) {
        size_t j = v.find(',', i);
        if (j == std::string::npos) j = v.size();
        out.push_back(parse_u64(flag, v.substr(i, j - i)));
        i = j + 1;
    }
    return out;
}

Options parse(int argc, char** argv) {
    Options o;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        std::string val;
        bool has_val = false;
        if (a.rfind("--", 0) == 0 && a.find('=') != std::string::npos) {
            val = a.substr(a.find('=') + 1);
            a = a.substr(0, a.find('='));
            has_val = true;
        }
        auto need = [&](const std::string& flag) -> std::string {
            if (has_val) return val;
            if (i + 1 >= argc) usage_error("a value is required for '" + flag + "'");
            return argv[++i];
        };
        if (a == "-h" || a == "--help") {
            print_help();
            std::exit(0);
        } else if (a == "--segregation") {
            std::string v = need(a);
            if (v == "deterministic") o.segregation = ECDNA_SEG_DETERMINISTIC;
            else if (v == "binomial") o.segregation = ECDNA_SEG_BINOMIAL;
            else if (v == "binomial-no-uneven") o.segregation = ECDNA_SEG_BINOMIAL_NO_UNEVEN;
            else if (v == "binomial-no-nminus") o.segregation = ECDNA_SEG_BINOMIAL_NO_NMINUS;
            else usage_error("invalid value '" + v + "' for '--segregation <SEGREGATION>'");
            o.segregation_name = v;
        } else if (a == "--growth") {
            o.growth = need(a);
            if (o.growth != "exponential" && o.growth != "constant")
                usage_error("invalid value '" + o.growth + "' for '--growth <GROWTH>'");
        } else if (a == "--b0") {
            o.b0_arg = need(a);
            o.b0 = parse_f32(a, o.b0_arg);
        } else if (a == "--b1") {
            o.b1_arg = need(a);
            o.b1 = parse_f32(a, o.b1_arg);
        } else if (a == "--d0") {
            o.d0_arg = need(a);
            o.d0 = parse_f32(a, o.d0_arg);
            o.has_d0 = true;
        } else if (a == "--d1") {
            o.d1_arg = need(a);
            o.d1 = parse_f32(a, o.d1_arg);
            o.has_d1 = true;
        } else if (a == "-y" || a == "--years") {
            o.years = parse_u64(a, need(a));
            o.has_years = true;
        } else if (a == "-c" || a == "--cells") {
            o.cells = parse_u64(a, need(a));
            o.has_cells = true;
        } else if (a == "--seed") {
            o.seed = parse_u64(a, need(a));
        } else if (a == "-d" || a == "--debug") {
            o.debug = true;
        } else if (a == "-s" || a == "--sequential") {
            o.sequential = true;
        } else if (a == "--initial") {
            o.initial = need(a);
            if (o.initial.size() < 5 || o.initial.substr(o.initial.size() - 5) != ".json")
                usage_error("invalid value '" + o.initial + "' for '--initial <FILE>': Must be JSON file: "
                            "extension must be .json)");
        } else if (a == "-r" || a == "--runs") {
            o.runs = parse_u64(a, need(a));
            o.has_runs = true;
        } else if (a == "--subsamples") {
            if (!has_val) usage_error("equal sign is needed when assigning values to '--subsamples=<N,...>'");
            o.subsamples = parse_list(a, val);
        } else if (a == "--snapshots") {
            if (!has_val) usage_error("equal sign is needed when assigning values to '--snapshots=<N,...>'");
            o.snapshots = parse_list(a, val);
            o.has_snapshots = true;
        } else if (a == "-v" || a == "--verbosity") {
            o.verbosity += 1;
        } else if (a.size() > 2 && a[0] == '-' && a[1] == 'v' && a.find_first_not_of('v', 1) == std::string::npos) {
            o.verbosity += (int)a.size() - 1;
        } else if (a == "--gpus") {
            o.gpus = (int)parse_u64(a, need(a));
            if (o.gpus < 1) usage_error("--gpus must be >= 1");
        } else if (a == "--time") {
            std::string v = need(a);
            if (v != "f32" && v != "f64") usage_error("--time must be f32 or f64");
            o.time_f64 = v == "f64";
        } else if (a == "--cell-cap") {
            o.cell_cap = parse_u64(a, need(a));
        } else if (a == "--hist-bins") {
            o.hist_bins = (uint32_t)parse_u64(a, need(a));
        } else if (a == "--dry-run") {
            o.dry_run = true;
        } else if (a == "--cell-store") {
            const std::string v = need(a);
            if (v != "bins" && v != "rows") usage_error("--cell-store must be bins or rows");
            o.rows = v == "rows";
            o.has_cell_store = true;
        } else if (a == "--bin-kmax") {
            const uint64_t v = parse_u64(a, need(a));
            if (v != 64 && v != 256) usage_error("--bin-kmax must be 64 or 256");
            o.bin_kmax = (uint32_t)v;
            o.has_bin_kmax = true;
        } else if (a == "--draws") {
            const std::string v = need(a);
            if (v != "philox" && v != "reference") usage_error("--draws must be philox or reference");
            o.reference_draws = v == "reference";
        } else if (a == "--pooled") {
            o.pooled = need(a);
        } else if (!a.empty() && a[0] == '-') {
            usage_error("unexpected argument '" + a + "' found");
        } else {
            pos.push_back(a);
        }
    }
    if (pos.size() != 1) usage_error(pos.empty() ? "the following required arguments were not provided: <DIR>"
                                                 : "unexpected argument '" + pos[1] + "' found");
    o.path = pos[0];
    // clap: `years` and `cells` share the group "stop"; debug conflicts with years, cells, sequential,
    // runs and verbosity (src/clap_app.rs:57-99)
    if (o.has_years && o.has_cells)
        usage_error("the argument '--years <YEARS>' cannot be used with '--cells <CELLS>'");
    if (o.debug && (o.has_years || o.has_cells || o.sequential || o.has_runs || o.verbosity))
        usage_error("the argument '--debug' cannot be used with the other run options");
    // the reference's draws address cells in swap_remove order: the row store, never the bins
    if (o.reference_draws && ((o.has_cell_store && !o.rows) || o.has_bin_kmax))
        usage_error("the argument '--draws reference' cannot be used with '--cell-store bins' or '--bin-kmax'");
    if (o.reference_draws) o.rows = true;
    // The engine's rate range (include/ecdna_ssa.h, since ABI v8): 0 or [2^-60, 2^60]; a divergence from the
    // reference, which takes any f32. Reported here as a usage error, before any GPU work.
    // (the message echoes the argument as given: std::to_string prints 6 fixed decimals, "1e-20" as "0.000000")
    struct RateArg {
        const char* flag;
        float value;
        const std::string* text;
    };
    const RateArg rate_args[] = {{"--b0 <RATE>", o.b0, &o.b0_arg}, {"--b1 <RATE>", o.b1, &o.b1_arg},
                                 {"--d0 <RATE>", o.d0, &o.d0_arg}, {"--d1 <RATE>", o.d1, &o.d1_arg}};
    for (const auto& ra : rate_args)
        if (!(ra.value == 0.f || (ra.value >= 0x1p-60f && ra.value <= 0x1p60f)))
            usage_error("invalid value '" + *ra.text + "' for '" + ra.flag +
                        "': rates must be 0 or in [2^-60, 2^60] (8.67e-19 .. 1.15e18) for this engine");
    return o;
}

// Cli::build (src/clap_app.rs:137-229)
struct Resolved {
    uint64_t cells, years, runs;
    int verbosity;
    bool parallel;
    bool birth_death;
    float d0, d1;
    std::vector<uint64_t> snapshots;
    Distribution initial;
    uint64_t cell_cap;
};

Resolved resolve(const Options& o) {
    Resolved r{};
    if (o.debug) {
        r.cells = 300;
        r.years = 2;
        r.verbosity = 255;
        r.parallel = false;
        r.runs = 1;
    } else if (o.has_years) {
        r.cells = kMaxCells;
        r.years = o.years;
        r.verbosity = o.verbosity;
        r.parallel = !o.sequential;
        r.runs = o.runs;
    } else {
        r.cells = o.has_cells ? o.cells : 1000;
        r.years = (uint64_t)(std::log2((float)r.cells) + 4.0f);  // (f32::log2(cells as f32) + 4f32) as u64
        r.verbosity = o.verbosity;
        r.parallel = !o.sequential;
        r.runs = o.runs;
    }
    r.snapshots = o.has_snapshots ? o.snapshots : ecdna::host::default_snapshots(r.cells);
    std::sort(r.snapshots.begin(), r.snapshots.end());
    const bool bd0 = o.has_d0 && o.d0 > 0.f, bd1 = o.has_d1 && o.d1 > 0.f;
    r.birth_death = bd0 || bd1;
    r.d0 = o.has_d0 ? o.d0 : 0.f;
    r.d1 = o.has_d1 ? o.d1 : 0.f;
    if (!o.initial.empty()) {
        r.initial = ecdna::host::load_json(o.initial);
    } else {
        r.initial.nplus = {1};  // {1: 1}, src/clap_app.rs:188-191
    }
    r.cell_cap = o.cell_cap ? o.cell_cap : (o.has_years ? (1ull << 24) : r.cells);
    r.cell_cap = std::max<uint64_t>(r.cell_cap, r.initial.nplus.size());
    return r;
}

std::string json_list(const std::vector<uint64_t>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
    return s + "]";
}

std::string now_str() {
    std::time_t t = std::time(nullptr);
    char buf[64];
    std::strftime(buf, sizeof(buf), "%Y-%m-%d %H:%M:%S UTC", std::gmtime(&t));
    return buf;
}

const char* stop_name(uint32_t s) {
    static const char* n[] = {"None", "MaxCellsReached", "MaxTimeReached", "MaxItersReached",
                              "AbsorbingStateReached", "Error"};
    return s < 6 ? n[s] : "?";
}

// Replicate shard g of `gpus`: [runs g / gpus, runs (g + 1) / gpus) — the contiguous split of
// ecdna_evo_amd.shard.shard_range (tests/test_host.py checks the two agree).
void shard_of(uint64_t runs, int gpus, int g, uint64_t& first, uint64_t& n) {
    first = runs * (uint64_t)g / (uint64_t)gpus;
    n = runs * (uint64_t)(g + 1) / (uint64_t)gpus - first;
}

struct Shard {
    int device;
    uint64_t first, n;
    void* comm = nullptr;  // RCCL communicator of this device (--pooled), or null
    std::vector<uint64_t> hist;
    std::vector<ecdna_totals_t> totals;
    std::vector<ecdna_rep_summary_t> summ;
    std::vector<uint16_t> rows;
    std::vector<ecdna_snapshot_t> snap_meta;
    std::vector<uint16_t> snap_rows;
    std::vector<uint64_t> rng_words;  // --draws reference: each replicate's ChaCha8 position at its end
    int64_t stride = 0;
    int rc = 0;
    std::string err;
};

void run_shard(const ecdna_ssa_params_t& base, Shard& sh, ecdna::host::Rendezvous* rv) {
    ecdna_ssa_params_t p = base;
    p.device = sh.device;
    p.first_replicate = sh.first;
    p.n_replicates = sh.n;
    ecdna_ssa_ctx* c = nullptr;
    sh.rc = ecdna_ssa_ctx_create(&p, &c);
    if (!sh.rc) sh.rc = ecdna_ssa_ctx_launch(c, nullptr);
    if (!sh.rc) {
        sh.stride = ecdna_ssa_ctx_row_stride(c);
        if (sh.stride <= 0) {
            sh.rc = ECDNA_E_NOMEM;
            sh.err = "the run does not fit in one device chunk; lower --runs or --cell-cap";
        }
    }
    if (!sh.rc) {
        sh.summ.resize(sh.n);
        sh.rows.resize(sh.n * (uint64_t)sh.stride);
        sh.rc = ecdna_ssa_ctx_download(c, sh.summ.data(), nullptr, nullptr, sh.rows.data());
    }
    if (!sh.rc && p.n_snapshots) {
        sh.snap_meta.resize(sh.n * p.n_snapshots);
        const uint64_t st = (p.cell_cap + 63) / 64 * 64;
        sh.snap_rows.resize(sh.n * p.n_snapshots * st);
        sh.rc = ecdna_ssa_ctx_download_snapshots(c, sh.snap_meta.data(), sh.snap_rows.data());
    }
    if (!sh.rc && (p.flags & ECDNA_FLAG_REFERENCE_DRAWS)) {  // where each replicate's rng stands (subsampling)
        sh.rng_words.resize(sh.n);
        sh.rc = ecdna_ssa_ctx_download_rng_words(c, sh.rng_words.data());
    }
    if (rv) {  // --pooled: the run's histogram and totals, all-reduced over the devices' shards (RCCL)
        const int rc = ecdna::host::join_reduction(*rv, sh.rc, [&] {
            int q = ecdna_ssa_ctx_reduce(c, sh.comm);
            sh.hist.resize((uint64_t)p.n_param_sets * p.hist_bins);
            sh.totals.resize(p.n_param_sets);
            if (!q) q = ecdna_ssa_ctx_download(c, nullptr, sh.hist.data(), sh.totals.data(), nullptr);
            return q;
        });
        if (!sh.rc && rc == ecdna::host::kPeerFailed) {
            sh.rc = ECDNA_E_STATE;
            sh.err = "another device's shard failed; no reduction";
        } else if (!sh.rc) {
            sh.rc = rc;
        }
    }
    if (sh.rc && sh.err.empty()) sh.err = ecdna_ssa_last_error_message();
    if (c) ecdna_ssa_ctx_destroy(c);
}

}  // namespace

int main(int argc, char** argv) {
    Options o = parse(argc, argv);
    Resolved r;
    try {
        r = resolve(o);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    if (o.growth == "constant") {  // GrowthOptions::Constant => todo!() (src/main.rs:49)
        std::fprintf(stderr, "error: --growth constant is not implemented (src/main.rs:49 is todo!())\n");
        return 1;
    }
    const uint64_t years_cap = r.years;
    // shards: one per GPU (sequential / debug: one; never more shards than replicates, so that every device
    // of the reduction has a shard)
    const int planned_gpus = (int)std::max<uint64_t>(1, std::min<uint64_t>(r.parallel ? o.gpus : 1, r.runs));
    std::string shards_json = "[";
    for (int g = 0; g < planned_gpus; ++g) {
        uint64_t f, n;
        shard_of(r.runs, planned_gpus, g, f, n);
        shards_json += (g ? ",[" : "[") + std::to_string(f) + "," + std::to_string(n) + "]";
    }
    shards_json += "]";
    if (o.dry_run) {
        std::printf(
            "{\"process\":\"%s\",\"segregation\":\"%s\",\"b0\":%.9g,\"b1\":%.9g,\"d0\":%.9g,\"d1\":%.9g,\"cells\":%llu,"
            "\"years\":%llu,\"runs\":%llu,\"seed\":%llu,\"verbosity\":%d,\"parallel\":%s,\"snapshots\":%s,"
            "\"subsamples\":%s,\"initial\":%s,\"cell_cap\":%llu,\"first_idx\":%llu,\"max_iter\":%llu,"
            "\"time\":\"%s\",\"gpus\":%d,\"cell_store\":\"%s\",\"bin_kmax\":%u,\"draws\":\"%s\",\"shards\":%s}\n",
            r.birth_death ? "BirthDeath" : "PureBirth", o.segregation_name.c_str(), (double)o.b0, (double)o.b1,
            (double)r.d0, (double)r.d1, (unsigned long long)r.cells,
            (unsigned long long)years_cap, (unsigned long long)r.runs, (unsigned long long)o.seed, r.verbosity,
            r.parallel ? "true" : "false", json_list(r.snapshots).c_str(), json_list(o.subsamples).c_str(),
            ecdna::host::to_json(r.initial).c_str(), (unsigned long long)r.cell_cap,
            (unsigned long long)(o.seed * 10), (unsigned long long)kMaxIter, o.time_f64 ? "f64" : "f32", o.gpus,
            o.rows ? "rows" : "bins", o.bin_kmax, o.reference_draws ? "reference" : "philox", shards_json.c_str());
        return 0;
    }

    if (ecdna_ssa_device_count() < 1) {  // no CPU fallback
        std::fprintf(stderr, "error: %s\n", ecdna_ssa_strerror(ECDNA_E_NODEVICE));
        return 1;
    }
    std::printf("%s Starting the simulation\n", now_str().c_str());  // src/main.rs:53
    ecdna_rates_t rates{o.b0, o.b1, r.d0, r.d1};
    ecdna_ssa_params_t p{};
    p.process = r.birth_death ? ECDNA_BIRTH_DEATH : ECDNA_PURE_BIRTH;
    p.segregation = o.segregation;
    p.rates = &rates;
    p.n_param_sets = 1;
    p.hist_bins = o.hist_bins;
    p.reps_per_set = std::max<uint64_t>(r.runs, 1);
    p.seed = o.seed;
    p.max_cells = r.cells;
    p.max_time = (double)(float)years_cap;  // `years as f32`, src/clap_app.rs:205
    p.max_iter = kMaxIter;
    p.cell_cap = (uint32_t)std::min<uint64_t>(r.cell_cap, 0xffffffffull);
    p.flags = (o.time_f64 ? 0u : ECDNA_FLAG_TIME_F32) | ECDNA_FLAG_SNAPSHOT_ROWS | (o.rows ? 0u : ECDNA_FLAG_BIN_STORE) |
              (o.reference_draws ? ECDNA_FLAG_REFERENCE_DRAWS : 0u);
    p.bin_kmax = o.rows ? 0u : o.bin_kmax;
    p.init_copies = r.initial.nplus.empty() ? nullptr : r.initial.nplus.data();
    p.init_nplus = (uint32_t)r.initial.nplus.size();
    p.init_nminus = r.initial.nminus;
    p.snapshot_cells = r.snapshots.data();
    p.n_snapshots = (uint32_t)r.snapshots.size();

    const int avail = ecdna_ssa_device_count();
    if (avail < 1) {
        std::fprintf(stderr, "error: %s\n", ecdna_ssa_strerror(ECDNA_E_NODEVICE));
        return 1;
    }
    const int gpus = std::min(planned_gpus, avail);
    std::vector<Shard> shards(gpus);
    for (int g = 0; g < gpus; ++g) {
        shards[g].device = g;
        shard_of(r.runs, gpus, g, shards[g].first, shards[g].n);
    }
    ecdna::host::Rendezvous rv;
    rv.total = gpus;
    std::vector<void*> comms;
    if (!o.pooled.empty() && r.runs) {  // one RCCL communicator per device (ncclCommInitAll)
        std::vector<int> devs(gpus);
        for (int g = 0; g < gpus; ++g) devs[g] = g;
        comms.assign(gpus, nullptr);
        if (int rc = ecdna_ssa_comm_init_all(gpus, devs.data(), comms.data())) {
            std::fprintf(stderr, "error: %s (%s)\n", ecdna_ssa_strerror(rc), ecdna_ssa_last_error_message());
            return 1;
        }
        for (int g = 0; g < gpus; ++g) shards[g].comm = comms[g];
    }
    ecdna::host::Rendezvous* rvp = comms.empty() ? nullptr : &rv;
    std::vector<std::thread> th;
    for (int g = 1; g < gpus; ++g)
        if (shards[g].n) th.emplace_back(run_shard, std::cref(p), std::ref(shards[g]), rvp);
    if (shards[0].n) run_shard(p, shards[0], rvp);
    for (auto& t : th) t.join();
    for (void* cm : comms) ecdna_ssa_comm_destroy(cm);
    for (auto& sh : shards) {
        if (sh.rc) {
            std::fprintf(stderr, "error on device %d: %s (%s)\n", sh.device, ecdna_ssa_strerror(sh.rc),
                         sh.err.c_str());
            return 1;
        }
    }

    const uint64_t snap_stride = (p.cell_cap + 63) / 64 * 64;
    try {
        for (auto& sh : shards) {
            for (uint64_t i = 0; i < sh.n; ++i) {
                const uint64_t rep = sh.first + i;
                const uint64_t idx = o.seed * 10 + rep;  // src/main.rs:214
                const std::string filename =
                    r.birth_death ? ecdna::host::filename_birth_death(o.b0, o.b1, r.d0, r.d1, idx)
                                  : ecdna::host::filename_pure_birth(o.b0, o.b1, idx);
                const ecdna_rep_summary_t& s = sh.summ[i];
                if (s.error) {
                    // the reference panics here (src/proliferation.rs:63-67 / src/process.rs:88)
                    std::fprintf(stderr, "replicate %llu: error %u, stopped after %llu iterations\n",
                                 (unsigned long long)idx, s.error, (unsigned long long)s.iters);
                }
                for (uint32_t q = 0; q < p.n_snapshots; ++q) {  // snapshots (src/process.rs:122-145)
                    const ecdna_snapshot_t& m = sh.snap_meta[i * p.n_snapshots + q];
                    if (!m.taken) continue;
                    Distribution d;
                    d.nminus = m.nminus;
                    const uint16_t* row = sh.snap_rows.data() + (i * p.n_snapshots + q) * snap_stride;
                    d.nplus.assign(row, row + m.nplus);
                    std::string path = ecdna::host::save(o.path, filename, (float)m.time, d);
                    if (r.verbosity > 0)
                        std::printf("saving state for timepoint at time %g with %llu cells in %s\n", m.time,
                                    (unsigned long long)d.cells(), path.c_str());
                }
                Distribution fin;  // end of the simulation (src/main.rs:100-109)
                fin.nminus = s.nminus;
                const uint16_t* row = sh.rows.data() + i * (uint64_t)sh.stride;
                fin.nplus.assign(row, row + s.nplus);
                ecdna::host::save(o.path, filename, (float)s.time, fin);
                // subsamples (src/main.rs:110-123, 184-197): under --draws reference with the replicate's own ChaCha8
                // stream, continued where the run left it and chained from one subsample to the next, as the
                // reference's `into_subsampled(*nb_cells, &mut rng)` loop does; else from a Philox region of the
                // replicate's key that the stepper never touches
                uint64_t word_pos = o.reference_draws ? sh.rng_words[i] : 0;
                for (size_t k = 0; k < o.subsamples.size(); ++k) {
                    Distribution sub = o.reference_draws
                                           ? ecdna::host::subsample_reference(fin, o.subsamples[k], o.seed, idx, word_pos)
                                           : ecdna::host::subsample(fin, o.subsamples[k], o.seed, rep, (uint32_t)k);
                    ecdna::host::save(o.path, filename, (float)s.time, sub);
                }
                if (r.verbosity > 0)  // src/main.rs:205-210
                    std::printf("stop reason: %s\nnminus, nplus: [%llu, %llu]\ntime: %g\n", stop_name(s.stop_reason),
                                (unsigned long long)s.nminus, (unsigned long long)s.nplus, s.time);
            }
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    if (!o.pooled.empty()) {  // every shard holds the reduced sums
        if (shards[0].hist.empty()) {  // --runs 0: nothing ran, an empty pool (there is always one shard)
            shards[0].hist.assign(p.hist_bins, 0);
            shards[0].totals.assign(1, ecdna_totals_t{});
        }
        const ecdna_totals_t& t = shards[0].totals[0];
        std::string js = "{\"histogram\":{";
        bool first = true;
        for (uint32_t b = 0; b < p.hist_bins; ++b) {
            if (!shards[0].hist[b]) continue;
            js += (first ? "\"" : ",\"") + std::to_string(b) + "\":" + std::to_string(shards[0].hist[b]);
            first = false;
        }
        js += "},\"overflow_bin\":" + std::to_string(p.hist_bins - 1) + ",\"replicates\":" + std::to_string(t.replicates) +
              ",\"events\":" + std::to_string(t.events) + ",\"nminus\":" + std::to_string(t.nminus) +
              ",\"nplus\":" + std::to_string(t.nplus) + ",\"errors\":" + std::to_string(t.errors) +
              ",\"stop_reasons\":[";
        for (int k = 0; k < 6; ++k) js += (k ? "," : "") + std::to_string(t.stop_reasons[k]);
        js += "],\"gpus\":" + std::to_string(gpus) + "}\n";
        FILE* f = std::fopen(o.pooled.c_str(), "w");
        if (!f || std::fputs(js.c_str(), f) < 0 || std::fclose(f) != 0) {
            std::fprintf(stderr, "error: cannot write %s\n", o.pooled.c_str());
            return 1;
        }
    }
    std::printf("%s End simulation\n", now_str().c_str());  // src/main.rs:226
    return 0;
}
