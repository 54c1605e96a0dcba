// aql_probe.hip — host cost of one kernel dispatch through the HIP runtime vs an AQL packet written
// to an HSA queue by this thread (gfx950, ROCm 7.2), and how fast the GPU drains back-to-back
// dispatches either way.  An empty kernel taking a 1.3 KiB argument struct (the node pass's
// K1Args + K1Step), 391 workgroups x 256; N dispatches round-robin over 4 streams / 4 queues.
// The AQL path finds the kernel HIP loaded (HSA loader extension: the process's executables and
// their symbols), writes each dispatch's arguments into a ring of host-pinned kernarg slots and
// the packet into the queue (header last, release), then rings the doorbell.
//   hipcc --offload-arch=gfx950 -O2 tools/aql_probe.hip -L/opt/rocm/lib -lhsa-runtime64 -o tools/bin_aql_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

struct Arg {
    unsigned char b[1344];
};
extern "C" __global__ void crane_probe_empty(Arg a) {
    // every argument dword is read (as the engine's kernels read theirs), nothing is written
    unsigned s = 0;
    for (int i = 0; i < (int)sizeof(Arg) / 4; ++i) s += reinterpret_cast<const unsigned*>(a.b)[i];
    if (s == 0x12345u && threadIdx.x == 999) asm volatile("s_nop 0");
}

#define HSA_OK(x)                                                                   \
    do {                                                                            \
        hsa_status_t s_ = (x);                                                      \
        if (s_ != HSA_STATUS_SUCCESS) {                                             \
            const char* m_ = nullptr;                                               \
            hsa_status_string(s_, &m_);                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?"); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

struct Found {
    hsa_agent_t agent{};
    const char* name = nullptr;
    uint64_t kobj = 0;
    uint32_t karg = 0, group = 0, priv = 0;
};

static hsa_status_t find_gpu(hsa_agent_t a, void* d) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        *static_cast<hsa_agent_t*>(d) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
    Found* f = static_cast<Found*>(d);
    hsa_symbol_kind_t k;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &k);
    if (k != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string nm(len, '\0');
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, nm.data());
    const std::string want = f->name;
    if (nm != want && nm != want + ".kd") return HSA_STATUS_SUCCESS;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &f->kobj);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &f->karg);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &f->group);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &f->priv);
    return HSA_STATUS_INFO_BREAK;
}

static hsa_ven_amd_loader_1_03_pfn_t g_ld;

static hsa_status_t find_cpu(hsa_agent_t a, void* d) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU) {
        *static_cast<hsa_agent_t*>(d) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t find_coarse(hsa_amd_memory_pool_t p, void* d) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t fl = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
    bool ok = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &ok);
    if (ok && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
        *static_cast<hsa_amd_memory_pool_t*>(d) = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t on_exe(hsa_executable_t e, void* d) {
    Found* f = static_cast<Found*>(d);
    hsa_status_t s = hsa_executable_iterate_agent_symbols(e, f->agent, on_symbol, d);
    return f->kobj ? HSA_STATUS_INFO_BREAK : (s == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : s);
}

int main() {
    const int kN = 3000, kGrid = 391, kBs = 256, kQ = 4;
    hipStream_t st[kQ];
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Arg a{};
    // HIP: per-launch host cost and drain time
    auto hip_run = [&]() {
        for (int i = 0; i < 64; ++i)
            hipExtLaunchKernelGGL(crane_probe_empty, dim3(kGrid), dim3(kBs), 0, st[i % kQ], nullptr, nullptr, 0u, a);
        hipDeviceSynchronize();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < kN; ++i)
            hipExtLaunchKernelGGL(crane_probe_empty, dim3(kGrid), dim3(kBs), 0, st[i % kQ], nullptr, nullptr, 0u, a);
        const auto t1 = std::chrono::steady_clock::now();
        hipDeviceSynchronize();
        const auto t2 = std::chrono::steady_clock::now();
        std::printf("hip: host %.3f us per launch, drained %.3f us per launch\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / kN,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / kN);
    };
    hip_run();

    HSA_OK(hsa_init());
    Found f;
    f.name = "crane_probe_empty";
    if (hsa_iterate_agents(find_gpu, &f.agent) != HSA_STATUS_INFO_BREAK) {
        std::fprintf(stderr, "no GPU agent\n");
        return 1;
    }
    size_t tsz = sizeof(g_ld);
    HSA_OK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, tsz, &g_ld));
    g_ld.hsa_ven_amd_loader_iterate_executables(on_exe, &f);
    if (!f.kobj) {
        std::fprintf(stderr, "kernel object not found\n");
        return 1;
    }
    std::printf("kernel object 0x%llx kernarg %u group %u private %u\n", (unsigned long long)f.kobj, f.karg, f.group,
                f.priv);
    if (f.karg < sizeof(Arg)) {
        std::fprintf(stderr, "kernarg segment smaller than the argument\n");
        return 1;
    }
    hsa_queue_t* q[kQ];
    hsa_signal_t done[kQ];
    for (int j = 0; j < kQ; ++j) {
        HSA_OK(hsa_queue_create(f.agent, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q[j]));
        HSA_OK(hsa_signal_create(0, 0, nullptr, &done[j]));
    }
    const size_t kslot = (f.karg + 255) / 256 * 256, nslot = 4096;
    unsigned char* rings[3] = {nullptr, nullptr, nullptr};
    const char* rname[3] = {"host coherent", "host non-coherent", "device (BAR)"};
    if (hipHostMalloc(reinterpret_cast<void**>(&rings[0]), kslot * nslot, hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&rings[1]), kslot * nslot, hipHostMallocNonCoherent) != hipSuccess) {
        std::fprintf(stderr, "kernarg ring\n");
        return 1;
    }
    {
        hsa_agent_t cpu{};
        hsa_amd_memory_pool_t pool{};
        hsa_iterate_agents(find_cpu, &cpu);
        if (hsa_amd_agent_iterate_memory_pools(f.agent, find_coarse, &pool) == HSA_STATUS_INFO_BREAK) {
            void* p = nullptr;
            HSA_OK(hsa_amd_memory_pool_allocate(pool, kslot * nslot, 0, &p));
            HSA_OK(hsa_amd_agents_allow_access(1, &cpu, nullptr, p));
            rings[2] = static_cast<unsigned char*>(p);
        }
    }
    for (auto* r : rings)
        if (r) std::memset(r, 0, kslot * nslot);
    std::printf("device ring %s (written and read back from the host)\n", rings[2] ? "mapped" : "unavailable");
    const uint16_t hdr_fence = (uint16_t)((HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                          (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE) |
                                          (1 << HSA_PACKET_HEADER_BARRIER));
    size_t slot = 0;
    // a "step": three dispatches on one queue, headers stored in order, one doorbell at the end
    // (device ring: a store fence and a read back of the last argument before the doorbell)
    auto step = [&](int j, bool last, unsigned char* ring, bool dev) {
        hsa_queue_t* qq = q[j];
        const uint64_t idx0 = hsa_queue_add_write_index_relaxed(qq, 3);
        while (idx0 + 3 - hsa_queue_load_read_index_scacquire(qq) > qq->size) {
        }
        volatile unsigned char* lastka = nullptr;
        for (int k = 0; k < 3; ++k) {
            const uint64_t idx = idx0 + k;
            unsigned char* ka = ring + kslot * (slot++ % nslot);
            std::memcpy(ka, &a, sizeof(a));
            lastka = ka;
            auto* p = static_cast<hsa_kernel_dispatch_packet_t*>(qq->base_address) + (idx & (qq->size - 1));
            p->workgroup_size_x = kBs;
            p->workgroup_size_y = 1;
            p->workgroup_size_z = 1;
            p->reserved0 = 0;
            p->grid_size_x = (uint32_t)(kGrid * kBs);
            p->grid_size_y = 1;
            p->grid_size_z = 1;
            p->private_segment_size = f.priv;
            p->group_segment_size = f.group;
            p->kernel_object = f.kobj;
            p->kernarg_address = ka;
            p->reserved2 = 0;
            p->completion_signal = (last && k == 2) ? done[j] : hsa_signal_t{0};
        }
        if (dev) {
            __builtin_ia32_sfence();
            (void)lastka[sizeof(a) - 1];
        }
        for (int k = 0; k < 3; ++k) {
            auto* p = static_cast<hsa_kernel_dispatch_packet_t*>(qq->base_address) + ((idx0 + k) & (qq->size - 1));
            const uint32_t word = (uint32_t)(hdr_fence | (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE)) |
                                  ((uint32_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16);
            __atomic_store_n(reinterpret_cast<uint32_t*>(p), word, __ATOMIC_RELEASE);
        }
        hsa_signal_store_screlease(qq->doorbell_signal, (hsa_signal_value_t)(idx0 + 2));
    };
    const int kSteps = kN / 3;
    for (int rep = 0; rep < 2; ++rep) {
        for (int v = 0; v < 3; ++v) {
            if (!rings[v]) continue;
            for (int j = 0; j < kQ; ++j) hsa_signal_store_screlease(done[j], 1);
            const auto t0 = std::chrono::steady_clock::now();
            // (the ring holds nslot dispatches: kN < nslot, no slot is reused while a kernel may read it)
            for (int i = 0; i < kSteps; ++i) step(i % kQ, i >= kSteps - kQ, rings[v], v == 2);
            const auto t1 = std::chrono::steady_clock::now();
            for (int j = 0; j < kQ; ++j)
                hsa_signal_wait_scacquire(done[j], HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
            const auto t2 = std::chrono::steady_clock::now();
            std::printf("aql, kernargs in %s: host %.3f us per dispatch, drained %.3f us per dispatch\n", rname[v],
                        std::chrono::duration<double, std::micro>(t1 - t0).count() / (3 * kSteps),
                        std::chrono::duration<double, std::micro>(t2 - t0).count() / (3 * kSteps));
        }
        hip_run();
    }
    for (int j = 0; j < kQ; ++j) {
        hsa_queue_destroy(q[j]);
        hsa_signal_destroy(done[j]);
    }
    hipHostFree(rings[0]);
    hipHostFree(rings[1]);
    if (rings[2]) hsa_amd_memory_pool_free(rings[2]);
    hsa_shut_down();
    return 0;
}
