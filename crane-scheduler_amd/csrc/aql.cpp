// aql.cpp — user-mode AQL queues for the engine's kernels (aql.hpp, crane_queue_* in
// include/crane_dyn.h).  Host code over the HSA runtime (the layer under HIP): the queue,
// its completion signal and kernarg ring are ours; the kernels are the ones HIP loaded for
// this library, found by name among the process's loaded executables (HSA loader extension).
#include "aql.hpp"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <cxxabi.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/crane_dyn.h"

namespace crane {
thread_local crane_queue* tl_aql = nullptr;
}

namespace {

struct KInfo {
    uint64_t kobj = 0;
    uint32_t karg = 0, group = 0, priv = 0;
};

constexpr uint32_t kQueuePackets = 1024;   // packets per queue (a power of two)
constexpr size_t kSlotBytes = 4096;        // kernarg bytes per packet slot (explicit + implicit)

// the library's kernels per GPU agent: mangled and demangled names -> descriptor
std::mutex g_mu;
std::map<uint64_t, std::unordered_map<std::string, KInfo>> g_kernels;
hsa_ven_amd_loader_1_03_pfn_t g_loader;
bool g_loader_ok = false;

struct SymScan {
    hsa_agent_t agent;
    std::unordered_map<std::string, KInfo>* out;
};

hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
    SymScan* sc = static_cast<SymScan*>(d);
    hsa_symbol_kind_t k;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &k) != HSA_STATUS_SUCCESS ||
        k != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string nm(len, '\0');
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &nm[0]);
    if (nm.size() > 3 && nm.compare(nm.size() - 3, 3, ".kd") == 0) nm.resize(nm.size() - 3);
    if (nm.compare(0, 9, "_ZN5crane") != 0) return HSA_STATUS_SUCCESS;  // this library's kernels only
    KInfo ki;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ki.kobj);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ki.karg);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &ki.group);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &ki.priv);
    (*sc->out)[nm] = ki;
    int st = 0;
    char* dm = abi::__cxa_demangle(nm.c_str(), nullptr, nullptr, &st);
    if (dm) {
        (*sc->out)[dm] = ki;
        std::free(dm);
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t on_exe(hsa_executable_t e, void* d) {
    SymScan* sc = static_cast<SymScan*>(d);
    (void)hsa_executable_iterate_agent_symbols(e, sc->agent, on_symbol, d);
    return HSA_STATUS_SUCCESS;
}

// (under g_mu) the kernel table of an agent, rescanned on demand
const std::unordered_map<std::string, KInfo>& scan_kernels(hsa_agent_t agent, bool rescan) {
    auto& m = g_kernels[agent.handle];
    if (rescan || m.empty()) {
        m.clear();
        SymScan sc{agent, &m};
        if (g_loader_ok) g_loader.hsa_ven_amd_loader_iterate_executables(on_exe, &sc);
    }
    return m;
}

struct AgentFind {
    uint32_t domain, bdf;
    hsa_agent_t gpu{0}, cpu{0};
};

hsa_status_t on_agent(hsa_agent_t a, void* d) {
    AgentFind* f = static_cast<AgentFind*>(d);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f->cpu.handle) f->cpu = a;
    if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if (bdf == f->bdf && dom == f->domain && !f->gpu.handle) f->gpu = a;
    return HSA_STATUS_SUCCESS;
}

hsa_status_t on_pool(hsa_amd_memory_pool_t p, void* d) {
    hsa_amd_segment_t seg;
    if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t fl = 0;
    bool ok = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &ok);
    if (ok && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
        *static_cast<hsa_amd_memory_pool_t*>(d) = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

struct crane_queue {
    int device = -1;
    bool hsa_up = false;  // hsa_init succeeded (hsa_shut_down at destroy)
    int ring_kind = 0;  // 0: device memory the host writes through the BAR, 1: pinned host memory
    hsa_agent_t agent{0};
    hsa_queue_t* q = nullptr;
    hsa_signal_t sig{0};  // committed steps still running
    unsigned char* ring = nullptr;  // kernarg slot of packet i: ring + (i % kQueuePackets) * kSlotBytes
    uint64_t first = 0, next = 0;   // packets [first, next) written, not yet committed
    std::atomic<uint64_t> commits{0};  // commits so far (each adds one to sig, its last packet takes one)
    std::unordered_map<const void*, KInfo> kinfo;  // per host stub
    std::string err;
    std::mutex umu;
    std::vector<crane_dyn*> users;  // engines that put steps here (aql_add_user)

    hipError_t fail(hipError_t e, const std::string& m) {
        err = m;
        return e;
    }
};

namespace crane {

// The queue's run-time check of the hand-packed implicit arguments (aql_launch): a kernel that
// reads the grid and group dimensions HIP derives from them (hidden block counts and group sizes
// of code object v5) and counts its workgroups.  A runtime whose layout differs fails the queue's
// creation, and the group keeps HIP launches (its dispatch -1).
__global__ void k_aql_selfcheck(uint32_t* out) {
    if (threadIdx.x == 0 && threadIdx.y == 0 && threadIdx.z == 0) {
        atomicAdd(&out[6], 1u);
        if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
            out[0] = gridDim.x;
            out[1] = gridDim.y;
            out[2] = gridDim.z;
            out[3] = blockDim.x;
            out[4] = blockDim.y;
            out[5] = blockDim.z;
        }
    }
}

const char* aql_error(const crane_queue* q) { return q ? q->err.c_str() : "null queue"; }

void aql_add_user(crane_queue* q, crane_dyn* h) {
    std::lock_guard<std::mutex> l(q->umu);
    for (crane_dyn* u : q->users)
        if (u == h) return;
    q->users.push_back(h);
}

void aql_remove_user(crane_queue* q, crane_dyn* h) {
    std::lock_guard<std::mutex> l(q->umu);
    for (size_t i = 0; i < q->users.size(); ++i)
        if (q->users[i] == h) {
            q->users.erase(q->users.begin() + (long)i);
            return;
        }
}

static const KInfo* lookup(crane_queue* q, const void* fn) {
    auto it = q->kinfo.find(fn);
    if (it != q->kinfo.end()) return &it->second;
    const char* name = hipKernelNameRefByPtr(fn, nullptr);
    if (!name) return nullptr;
    std::lock_guard<std::mutex> l(g_mu);
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
            // not loaded yet: a HIP query of the function loads its code object, then rescan
            hipFuncAttributes fa;
            (void)hipFuncGetAttributes(&fa, fn);
        }
        const auto& m = scan_kernels(q->agent, pass == 1);
        auto k = m.find(name);
        if (k == m.end()) {
            std::string s(name);
            if (s.size() > 3 && s.compare(s.size() - 3, 3, ".kd") == 0) k = m.find(s.substr(0, s.size() - 3));
        }
        if (k != m.end()) return &(q->kinfo[fn] = k->second);
    }
    return nullptr;
}

static inline hsa_kernel_dispatch_packet_t* packet(crane_queue* q, uint64_t i) {
    return static_cast<hsa_kernel_dispatch_packet_t*>(q->q->base_address) + (i & (kQueuePackets - 1));
}

hipError_t aql_launch(crane_queue* q, const void* fn, dim3 grid, dim3 block, uint32_t dyn_lds,
                      const unsigned char* args, size_t explicit_bytes) {
    const KInfo* k = lookup(q, fn);
    if (!k) return q->fail(hipErrorInvalidDeviceFunction, "aql: kernel not found among the loaded code objects");
    if (k->karg > kSlotBytes || explicit_bytes > k->karg)
        return q->fail(hipErrorInvalidConfiguration, "aql: kernel argument segment too large");
    if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;  // (HIP launches nothing either)
    const uint64_t i = q->next;
    // the slot's previous packet (kQueuePackets ago) and its kernargs must be done: the packet
    // processor has moved 2 past it (each packet waits for the one before it: barrier bit)
    if (i + 2 > kQueuePackets) {
        if (q->first < q->next && hsa_queue_load_read_index_scacquire(q->q) + kQueuePackets < i + 2) {
            hipError_t e = aql_commit(q);  // (let the processor reach what this thread wrote)
            if (e != hipSuccess) return e;
        }
        // (bounded like aql_wait: a faulted or hung kernel is reported, not waited for forever)
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spins = 0; hsa_queue_load_read_index_scacquire(q->q) + kQueuePackets < i + 2; ++spins) {
            cpu_relax();
            if ((spins & 4095) == 4095 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                return q->fail(hipErrorLaunchTimeOut, "aql: the queue's packet ring did not drain within 60 s");
        }
    }
    unsigned char* ka = q->ring + (i & (kQueuePackets - 1)) * kSlotBytes;
    // the explicit arguments, then the code-object-v5 implicit ones the kernel may read, at
    // the 8-byte aligned end of the explicit ones (tests/test_aql.py checks every kernel's
    // metadata against this layout): block counts, group sizes, remainders (0: whole
    // groups), global offsets (0), grid dimensions, dynamic LDS size
    alignas(16) unsigned char img[kSlotBytes];
    std::memcpy(img, args, explicit_bytes);
    std::memset(img + explicit_bytes, 0, k->karg - explicit_bytes);
    const size_t base = (explicit_bytes + 7) & ~(size_t)7;
    auto put32 = [&](size_t o, uint32_t v) {
        if (base + o + 4 <= k->karg) std::memcpy(img + base + o, &v, 4);
    };
    auto put16 = [&](size_t o, uint16_t v) {
        if (base + o + 2 <= k->karg) std::memcpy(img + base + o, &v, 2);
    };
    put32(0, grid.x);
    put32(4, grid.y);
    put32(8, grid.z);
    put16(12, (uint16_t)block.x);
    put16(14, (uint16_t)block.y);
    put16(16, (uint16_t)block.z);
    put16(64, (uint16_t)(grid.z > 1 || block.z > 1 ? 3 : grid.y > 1 || block.y > 1 ? 2 : 1));
    put32(120, dyn_lds);
    std::memcpy(ka, img, (k->karg + 15) & ~(size_t)15);
    hsa_kernel_dispatch_packet_t* p = packet(q, i);
    p->workgroup_size_x = (uint16_t)block.x;
    p->workgroup_size_y = (uint16_t)block.y;
    p->workgroup_size_z = (uint16_t)block.z;
    p->reserved0 = 0;
    p->grid_size_x = grid.x * block.x;
    p->grid_size_y = grid.y * block.y;
    p->grid_size_z = grid.z * block.z;
    p->private_segment_size = k->priv;
    p->group_segment_size = k->group + dyn_lds;
    p->kernel_object = k->kobj;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    p->completion_signal = hsa_signal_t{0};
    q->next = i + 1;
    return hipSuccess;
}

hipError_t aql_commit(crane_queue* q) {
    if (q->first == q->next) return hipSuccess;
    const uint64_t last = q->next - 1;
    packet(q, last)->completion_signal = q->sig;
    hsa_signal_add_relaxed(q->sig, 1);
    q->commits.fetch_add(1, std::memory_order_release);
    if (q->ring_kind == 0) {
        // the kernargs went through write-combining BAR stores: fence them and read one back so
        // they are in device memory before the packet processor can fetch them
        __builtin_ia32_sfence();
        (void)*reinterpret_cast<volatile const uint32_t*>(q->ring + (last & (kQueuePackets - 1)) * kSlotBytes);
    }
    for (uint64_t i = q->first; i < q->next; ++i) {
        hsa_kernel_dispatch_packet_t* p = packet(q, i);
        const uint32_t dims = p->grid_size_z > 1 ? 3u : p->grid_size_y > 1 ? 2u : 1u;
        // agent-scope acquire and release on every packet: the inputs and outputs are device
        // memory read and written by this device (its kernels, copies and RCCL), and agent
        // scope is what makes one XCD's L2 contents visible to the others.  System scope on a
        // step's first and last packet (host-coherent visibility, which nothing here needs)
        // cost 4 us of a config-3 batch's latency and 0.0121 -> 0.0126 ms per batch in flight
        // (profiles/r05/dispatch_queue_ab.txt)
        const uint32_t acq = HSA_FENCE_SCOPE_AGENT, rel = HSA_FENCE_SCOPE_AGENT;
        const uint16_t hdr = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                        (1u << HSA_PACKET_HEADER_BARRIER) |
                                        (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                        (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
        const uint32_t word = (uint32_t)hdr | ((uint32_t)(dims << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16);
        __atomic_store_n(reinterpret_cast<uint32_t*>(p), word, __ATOMIC_RELEASE);
    }
    hsa_queue_store_write_index_screlease(q->q, q->next);
    hsa_signal_store_screlease(q->q->doorbell_signal, (hsa_signal_value_t)last);
    q->first = q->next;
    return hipSuccess;
}

uint64_t aql_commits(const crane_queue* q) { return q->commits.load(std::memory_order_acquire); }

uint64_t aql_completed(const crane_queue* q) {
    // (the signal counts the commits still running; read after the count so a commit between the
    // two reads makes the result smaller, never larger)
    const uint64_t c = q->commits.load(std::memory_order_acquire);
    const hsa_signal_value_t v = hsa_signal_load_scacquire(q->sig);
    return v <= 0 ? c : c - std::min<uint64_t>(c, (uint64_t)v);
}

hipError_t aql_wait(crane_queue* q) {
    hipError_t e = aql_commit(q);
    if (e != hipSuccess) return e;
    // (a bounded wait: a step that never finishes is reported, not waited for forever)
    const auto t0 = std::chrono::steady_clock::now();
    while (hsa_signal_wait_scacquire(q->sig, HSA_SIGNAL_CONDITION_EQ, 0, 1000000, HSA_WAIT_STATE_ACTIVE) != 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
            return q->fail(hipErrorLaunchTimeOut, "aql: steps on the queue did not finish within 60 s");
    }
    return hipSuccess;
}

}  // namespace crane

using namespace crane;

namespace {

// one launch of k_aql_selfcheck on the new queue over a 3-D grid; its readings must be the
// launch's own dimensions
int aql_selfcheck(crane_queue* q) {
    const dim3 grid(5, 3, 2), block(32, 2, 1);
    uint32_t* d = nullptr;
    uint32_t h[8] = {};
    if (hipMalloc(reinterpret_cast<void**>(&d), sizeof h) != hipSuccess) {
        q->err = "aql self-check: hipMalloc failed";
        return CRANE_E_HIP;
    }
    hipError_t e = hipMemset(d, 0, sizeof h);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned char args[8];
    size_t off = 0;
    aql_pack(args, off, d);
    if (e == hipSuccess) e = aql_launch(q, reinterpret_cast<const void*>(&k_aql_selfcheck), grid, block, 0, args, off);
    if (e == hipSuccess) e = aql_wait(q);
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) {
        if (q->err.empty()) q->err = std::string("aql self-check: ") + hipGetErrorString(e);
        return CRANE_E_HIP;
    }
    const uint32_t want[7] = {grid.x, grid.y, grid.z, block.x, block.y, block.z, grid.x * grid.y * grid.z};
    for (int i = 0; i < 7; ++i)
        if (h[i] != want[i]) {
            q->err = "aql self-check: implicit-argument layout differs from this runtime's (field " + std::to_string(i) +
                     ": " + std::to_string(h[i]) + ", want " + std::to_string(want[i]) + ")";
            return CRANE_E_HIP;
        }
    return CRANE_OK;
}

}  // namespace

extern "C" {

int crane_queue_create(int32_t device, int32_t ring_kind, crane_queue** out) {
    if (!out) return CRANE_E_INVALID;
    crane_queue* q = new crane_queue();
    *out = q;  // returned on failure too (its error is readable); destroy it either way
    if (ring_kind < 0 || ring_kind > 1) {
        q->err = "ring_kind: 0 (device memory) | 1 (pinned host memory)";
        return CRANE_E_INVALID;
    }
    q->device = device;
    q->ring_kind = ring_kind;
    int bus = 0, dv = 0, dom = 0;
    if (hipSetDevice(device) != hipSuccess || hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) ||
        hipDeviceGetAttribute(&dv, hipDeviceAttributePciDeviceId, device) ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, device)) {
        q->err = "device " + std::to_string(device) + " not visible";
        return CRANE_E_INVALID;
    }
    if (hsa_init() != HSA_STATUS_SUCCESS) {  // (reference-counted: HIP initialised it already)
        q->err = "hsa_init failed";
        return CRANE_E_HIP;
    }
    q->hsa_up = true;
    {
        std::lock_guard<std::mutex> l(g_mu);
        if (!g_loader_ok) {
            g_loader_ok = hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(g_loader),
                                                               &g_loader) == HSA_STATUS_SUCCESS;
        }
        if (!g_loader_ok) {
            q->err = "HSA loader extension unavailable";
            return CRANE_E_HIP;
        }
    }
    AgentFind f{(uint32_t)dom, (uint32_t)((bus << 8) | (dv << 3))};
    hsa_iterate_agents(on_agent, &f);
    if (!f.gpu.handle) {
        q->err = "no HSA agent for device " + std::to_string(device);
        return CRANE_E_HIP;
    }
    q->agent = f.gpu;
    if (hsa_queue_create(f.gpu, kQueuePackets, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX,
                         &q->q) != HSA_STATUS_SUCCESS) {
        q->q = nullptr;
        q->err = "hsa_queue_create failed";
        return CRANE_E_HIP;
    }
    if (hsa_signal_create(0, 0, nullptr, &q->sig) != HSA_STATUS_SUCCESS) {
        q->sig.handle = 0;
        q->err = "hsa_signal_create failed";
        return CRANE_E_HIP;
    }
    const size_t bytes = (size_t)kQueuePackets * kSlotBytes;
    if (ring_kind == 0) {
        hsa_amd_memory_pool_t pool{0};
        void* p = nullptr;
        if (hsa_amd_agent_iterate_memory_pools(f.gpu, on_pool, &pool) != HSA_STATUS_INFO_BREAK ||
            hsa_amd_memory_pool_allocate(pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) {
            q->err = "device kernarg ring: no allocation";
            return CRANE_E_HIP;
        }
        q->ring = static_cast<unsigned char*>(p);
        if (!f.cpu.handle || hsa_amd_agents_allow_access(1, &f.cpu, nullptr, p) != HSA_STATUS_SUCCESS) {
            q->err = "device kernarg ring: no host access";
            return CRANE_E_HIP;
        }
    } else if (hipHostMalloc(reinterpret_cast<void**>(&q->ring), bytes, hipHostMallocCoherent) != hipSuccess) {
        q->ring = nullptr;
        q->err = "pinned kernarg ring: no allocation";
        return CRANE_E_HIP;
    }
    std::memset(q->ring, 0, bytes);
    return aql_selfcheck(q);
}

int crane_queue_wait(crane_queue* q) {
    if (!q || !q->q) return CRANE_E_INVALID;
    return aql_wait(q) == hipSuccess ? CRANE_OK : CRANE_E_HIP;
}

const char* crane_queue_last_error(const crane_queue* q) { return aql_error(q); }

int crane_queue_destroy(crane_queue* q) {
    if (!q) return CRANE_OK;
    if (q->q && q->sig.handle) (void)aql_wait(q);
    // the engines that used the queue forget it (their next state change would wait on it)
    std::vector<crane_dyn*> us;
    {
        std::lock_guard<std::mutex> l(q->umu);
        us.swap(q->users);
    }
    for (crane_dyn* h : us) engine_drop_queue(h, q);
    if (q->q) hsa_queue_destroy(q->q);
    if (q->sig.handle) hsa_signal_destroy(q->sig);
    if (q->ring) {
        if (q->ring_kind == 0) hsa_amd_memory_pool_free(q->ring);
        else (void)hipHostFree(q->ring);
    }
    if (q->hsa_up) hsa_shut_down();
    delete q;
    return CRANE_OK;
}

}  // extern "C"
