// Host-side cost of one has_match before the first launch: record the
// reference's op DAG (parse + build_branches + Execution) and lower it to the
// PBS program.  g++ -O2 -std=c++17 -Iinclude -Ifhe-regex_amd/csrc tools/host_bench.cpp
//   fhe-regex_amd/build/{regex,merged,lower,capi,keys,fft}.o ... (see tools/host_bench.sh)
#include <chrono>
#include <cstdio>
#include <random>
#include <string>

#include "lower.h"
#include "regex.h"

using namespace fr;
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const std::string pat = argc > 1 ? argv[1] : "/abc/";
    const size_t L = argc > 2 ? (size_t)std::atoi(argv[2]) : 256;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 50;
    double tr = 0, tl = 0;
    size_t gates = 0;
    for (int it = 0; it < iters; ++it) {
        double t0 = ms();
        ValueDag dag;
        Recorded rec = record_has_match_engine(dag, L, pat, 0, L, FR_ENGINE_AUTO);
        double t1 = ms();
        Program prog = lower(dag, rec.root, FR_LOWER_THRESHOLD);
        double t2 = ms();
        tr += t1 - t0;
        tl += t2 - t1;
        gates = prog.gates.size();
    }
    std::printf("%s L=%zu: record %.3f ms, lower %.3f ms, %zu gates\n", pat.c_str(), L, tr / iters, tl / iters, gates);
}
