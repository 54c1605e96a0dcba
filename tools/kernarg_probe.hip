// kernarg_probe.hip — host enqueue cost of a kernel launch vs its kernel-argument size
// (gfx950, ROCm 7.2): an empty kernel taking a 16-byte vs a 1.3 KiB argument struct (the node
// pass's K1Args + K1Step), hipExtLaunchKernelGGL as the engine launches, N launches per stream
// round-robin over 4 streams; prints us per launch on the enqueuing thread.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int B>
struct Arg {
    unsigned char b[B];
};
template <int B>
__global__ void k_empty(Arg<B> a) {
    if (a.b[0] == 123 && threadIdx.x == 999) asm volatile("s_nop 0");
}

template <int B>
double run(hipStream_t* st, int n, int grid) {
    Arg<B> a{};
    for (int i = 0; i < 64; ++i) hipExtLaunchKernelGGL(k_empty<B>, dim3(grid), dim3(256), 0, st[i & 3], nullptr, nullptr, 0u, a);
    hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hipExtLaunchKernelGGL(k_empty<B>, dim3(grid), dim3(256), 0, st[i & 3], nullptr, nullptr, 0u, a);
    const auto t1 = std::chrono::steady_clock::now();
    hipDeviceSynchronize();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t st[4];
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int rep = 0; rep < 3; ++rep)
        std::printf("grid 391: 16 B %.2f us, 256 B %.2f us, 1344 B %.2f us, 3 KiB %.2f us per launch\n",
                    run<16>(st, 2000, 391), run<256>(st, 2000, 391), run<1344>(st, 2000, 391), run<3072>(st, 2000, 391));
    return 0;
}
