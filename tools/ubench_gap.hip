// Dependent-launch gap on one stream: K back-to-back launches of a tiny kernel (every one
// reading what the previous wrote), as plain launches, as launches carrying start/stop
// events (the profiling timers' form), and replayed from a captured hipGraph.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench_gap.hip -o tools/ubench_gap && tools/ubench_gap
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void k_step(unsigned long long* v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = v[i] * 6364136223846793005ull + 1442695040888963407ull;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int K = 2000, n = 256 * 256, grid = n / 256;
    unsigned long long* v;
    CK(hipMalloc(&v, n * 8));
    CK(hipMemset(v, 0, n * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned flags = argc > 1 ? (unsigned)strtoul(argv[1], nullptr, 0) : 0u;  // event flags
    std::vector<hipEvent_t> ev(2 * K);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, flags));
    printf("event flags 0x%x\n", flags);
    for (int rep = 0; rep < 3; ++rep) {
        // plain launches
        CK(hipStreamSynchronize(s));
        double t = now_us();
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, v, n);
        CK(hipStreamSynchronize(s));
        const double plain = (now_us() - t) / K;
        // launches with start/stop events
        t = now_us();
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, ev[2 * i], ev[2 * i + 1], 0, v, n);
        CK(hipStreamSynchronize(s));
        const double evd = (now_us() - t) / K;
        // only a stop event on every launch
        t = now_us();
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, nullptr, ev[2 * i + 1], 0, v, n);
        CK(hipStreamSynchronize(s));
        const double stopd = (now_us() - t) / K;
        // only a start event on every launch
        t = now_us();
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, ev[2 * i], nullptr, 0, v, n);
        CK(hipStreamSynchronize(s));
        const double startd = (now_us() - t) / K;
        // a stop event on every other launch (the chained-stop timer form: one per kernel timed)
        t = now_us();
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, nullptr, (i & 1) ? ev[2 * i + 1] : nullptr, 0,
                                  v, n);
        CK(hipStreamSynchronize(s));
        const double stop2d = (now_us() - t) / K;
        // graph replay
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, s, v, n);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));  // warm
        CK(hipStreamSynchronize(s));
        t = now_us();
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        const double graph = (now_us() - t) / K;
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        printf("per dependent launch (us): plain %.2f  start+stop events %.2f  stop event %.2f  start event %.2f  "
               "stop event on every other %.2f  graph %.2f\n",
               plain, evd, stopd, startd, stop2d, graph);
    }
    return 0;
}
