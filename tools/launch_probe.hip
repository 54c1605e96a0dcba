// Host cost of the ways to enqueue a 3-kernel step on one stream (no GPU work to
// speak of): 3 hipExtLaunchKernelGGL, hipLaunchKernel, a hipGraph of the 3 kernels,
// a small H2D hipMemcpyAsync.  Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o /tmp/lp
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

struct Big {
    char b[1168];
};
struct Small {
    char b[256];
};
__global__ void kbig(Big a, int* o) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[5] == 7) o[0] = 1;
}
__global__ void ksmall(Small a, int* o) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[5] == 7) o[0] = 1;
}

template <class F>
static double per_op_us(int n, F f, hipStream_t s) {
    for (int i = 0; i < 50; ++i) f();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* o;
    hipMalloc(&o, 64);
    Big big{};
    Small sm{};
    const int n = 300;
    auto ext3 = [&] {
        hipExtLaunchKernelGGL(ksmall, dim3(400), dim3(512), 0, s, nullptr, nullptr, 0u, sm, o);
        hipExtLaunchKernelGGL(kbig, dim3(400), dim3(256), 0, s, nullptr, nullptr, 0u, big, o);
        hipExtLaunchKernelGGL(ksmall, dim3(320), dim3(1024), 0, s, nullptr, nullptr, 0u, sm, o);
    };
    auto small3 = [&] {
        for (int k = 0; k < 3; ++k) hipExtLaunchKernelGGL(ksmall, dim3(400), dim3(256), 0, s, nullptr, nullptr, 0u, sm, o);
    };
    auto chev = [&] {
        hipLaunchKernelGGL(ksmall, dim3(400), dim3(512), 0, s, sm, o);
        hipLaunchKernelGGL(kbig, dim3(400), dim3(256), 0, s, big, o);
        hipLaunchKernelGGL(ksmall, dim3(320), dim3(1024), 0, s, sm, o);
    };
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    ext3();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    auto graph = [&] { hipGraphLaunch(ge, s); };
    long long hv[32] = {};
    long long* dv;
    hipMalloc(&dv, sizeof hv);
    long long* pinned;
    hipHostMalloc(&pinned, sizeof hv, 0);
    auto h2d = [&] { hipMemcpyAsync(dv, pinned, sizeof hv, hipMemcpyHostToDevice, s); };
    auto h2d_graph = [&] {
        hipMemcpyAsync(dv, pinned, sizeof hv, hipMemcpyHostToDevice, s);
        hipGraphLaunch(ge, s);
    };
    auto setdev = [&] { hipSetDevice(0); };
    auto lasterr = [&] { (void)hipGetLastError(); };
    printf("{\"ext3_mixed_us\": %.2f, \"ext3_small_us\": %.2f, \"launch3_us\": %.2f, \"graph3_us\": %.2f, "
           "\"h2d_256B_us\": %.2f, \"h2d_plus_graph_us\": %.2f, \"setdevice_us\": %.3f, \"getlasterror_us\": %.3f}\n",
           per_op_us(n, ext3, s), per_op_us(n, small3, s), per_op_us(n, chev, s), per_op_us(n, graph, s),
           per_op_us(n, h2d, s), per_op_us(n, h2d_graph, s), per_op_us(n, setdev, s), per_op_us(n, lasterr, s));
    // T host threads, each its own stream, 3 launches per step: aggregate host rate
    for (int T : {2, 4}) {
        std::vector<hipStream_t> ss(T);
        for (auto& x : ss) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        auto run = [&](int t) {
            for (int i = 0; i < n; ++i) {
                hipExtLaunchKernelGGL(ksmall, dim3(400), dim3(512), 0, ss[t], nullptr, nullptr, 0u, sm, o);
                hipExtLaunchKernelGGL(kbig, dim3(400), dim3(256), 0, ss[t], nullptr, nullptr, 0u, big, o);
                hipExtLaunchKernelGGL(ksmall, dim3(320), dim3(1024), 0, ss[t], nullptr, nullptr, 0u, sm, o);
            }
        };
        for (int w = 0; w < 2; ++w) {
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back(run, t);
            for (auto& x : th) x.join();
            auto t1 = std::chrono::steady_clock::now();
            hipDeviceSynchronize();
            if (w) printf("{\"threads\": %d, \"us_per_step_aggregate\": %.2f}\n", T,
                          std::chrono::duration<double, std::micro>(t1 - t0).count() / (n * T));
        }
    }
    return 0;
}
