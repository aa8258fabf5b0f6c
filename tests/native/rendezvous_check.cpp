// tests/native/rendezvous_check.cpp — host-only check of the multi-device --pooled rendezvous
// (ecdna::host::Rendezvous / join_reduction, ecdna-evo_amd/host/ecdna_host.hpp) with the RCCL reduction
// stubbed: N shard threads, some failing; the collective stub must run on every thread when all succeed and
// on none otherwise, and each thread's status must say why. Built and run by tests/test_host.py.
// Usage: rendezvous_check <ok flags, e.g. 1101>; prints "calls=<c> rc=<rc0>,<rc1>,..."
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "ecdna_host.hpp"

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    const std::string flags = argv[1];
    const int n = (int)flags.size();
    ecdna::host::Rendezvous rv;
    rv.total = n;
    std::atomic<int> calls{0};
    std::vector<int> rc(n, 0);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            const int own = flags[i] == '1' ? 0 : -2;  // a failed shard (e.g. ECDNA_E_HIP)
            std::this_thread::sleep_for(std::chrono::milliseconds(5 * (n - i)));  // arrive in reverse order
            rc[i] = ecdna::host::join_reduction(rv, own, [&] {
                calls.fetch_add(1);
                return 0;
            });
        });
    for (auto& t : th) t.join();
    std::printf("calls=%d rc=", calls.load());
    for (int i = 0; i < n; ++i) std::printf("%s%d", i ? "," : "", rc[i]);
    std::printf("\n");
    return 0;
}
