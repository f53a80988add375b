// Can the host write device memory directly (large-BAR mapping)?  If so, a persistent worker could take
// descriptors AND small-call input data from HBM instead of reading them over PCIe (one round trip each).
// Tries hipExtMallocWithFlags(fine-grained / uncached) and the HSA pool API with CPU access granted;
// reports the pointer attributes, checks CPU writes against a device read, and times CPU writes of 6 KiB.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 profiles/r03/persist/bar_probe.hip -lhsa-runtime64 -o profiles/r03/persist/bar_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <immintrin.h>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void sum_kernel(const unsigned* p, int n, unsigned* out) {
    unsigned s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    atomicAdd(out, s);
}

static void try_ptr(const char* name, void* p, size_t n) {
    hipPointerAttribute_t a{};
    hipError_t e = hipPointerGetAttributes(&a, p);
    printf("%s: ptr %p attr rc=%d type=%d device=%d hostPointer=%p devicePointer=%p\n", name, p, (int)e, (int)a.type,
           a.device, a.hostPointer, a.devicePointer);
    fflush(stdout);
}

static void time_writes(const char* name, unsigned* host_view, unsigned* dev_view) {
    const int n = 6 * 1024 / 4;
    std::vector<unsigned> src(n);
    for (int i = 0; i < n; i++) src[i] = i * 2654435761u;
    double best = 1e9;
    for (int r = 0; r < 2000; r++) {
        const double t0 = now();
        memcpy(host_view, src.data(), n * 4);
        _mm_sfence();
        const double t = now() - t0;
        if (t < best) best = t;
    }
    unsigned* out = nullptr;
    hipMalloc(&out, 4);
    hipMemset(out, 0, 4);
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, dev_view, n, out);
    unsigned got = 0;
    hipMemcpy(&got, out, 4, hipMemcpyDeviceToHost);
    unsigned want = 0;
    for (int i = 0; i < n; i++) want += src[i];
    // CPU read back (uncached reads over the BAR are slow; one pass)
    const double t0 = now();
    unsigned rb = 0;
    for (int i = 0; i < n; i++) rb += ((volatile unsigned*)host_view)[i];
    const double tr = now() - t0;
    printf("%s: CPU write 6 KiB + sfence best %.2f us; device sum %s; CPU read back 6 KiB %.2f us (%s)\n", name, best * 1e6,
           got == want ? "matches" : "DIFFERS", tr * 1e6, rb == want ? "ok" : "differs");
    fflush(stdout);
    hipFree(out);
}

int main() {
    hipSetDevice(0);
    for (unsigned flag : {hipDeviceMallocFinegrained, hipDeviceMallocUncached}) {
        void* p = nullptr;
        hipError_t e = hipExtMallocWithFlags(&p, 1 << 20, flag);
        printf("hipExtMallocWithFlags(flag %u) rc=%d\n", flag, (int)e);
        if (e == hipSuccess) try_ptr("  hip", p, 1 << 20);
    }
    // HSA: the GPU agent's pools; allocate in a pool allowed for the CPU
    hsa_init();
    struct Ctx {
        hsa_agent_t cpu{}, gpu{};
        bool have_cpu = false, have_gpu = false;
    } c;
    hsa_iterate_agents([](hsa_agent_t a, void* d) {
        Ctx& c = *(Ctx*)d;
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_CPU && !c.have_cpu) { c.cpu = a; c.have_cpu = true; }
        if (t == HSA_DEVICE_TYPE_GPU && !c.have_gpu) { c.gpu = a; c.have_gpu = true; }
        return HSA_STATUS_SUCCESS;
    }, &c);
    struct Pools { std::vector<hsa_amd_memory_pool_t> v; } pools;
    hsa_amd_agent_iterate_memory_pools(c.gpu, [](hsa_amd_memory_pool_t p, void* d) {
        ((Pools*)d)->v.push_back(p);
        return HSA_STATUS_SUCCESS;
    }, &pools);
    for (size_t i = 0; i < pools.v.size(); i++) {
        hsa_amd_memory_pool_t pool = pools.v[i];
        hsa_amd_segment_t seg;
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
        uint32_t flags = 0;
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
        bool alloc = false;
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
        hsa_amd_memory_pool_access_t acc;
        hsa_amd_agent_memory_pool_get_info(c.cpu, pool, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
        printf("gpu pool %zu: segment %d global_flags 0x%x alloc %d cpu_access %d\n", i, (int)seg, flags, (int)alloc, (int)acc);
        if (seg != HSA_AMD_SEGMENT_GLOBAL || !alloc) continue;
        void* p = nullptr;
        hsa_status_t s = hsa_amd_memory_pool_allocate(pool, 1 << 20, 0, &p);
        if (s != HSA_STATUS_SUCCESS) { printf("  allocate failed %d\n", (int)s); continue; }
        s = hsa_amd_agents_allow_access(1, &c.cpu, nullptr, p);
        printf("  allocated %p, allow CPU access rc=%d\n", p, (int)s);
        fflush(stdout);
        hsa_agent_t both[2] = {c.gpu, c.cpu};
        hsa_amd_agents_allow_access(2, both, nullptr, p);
        if (s == HSA_STATUS_SUCCESS && acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED) {
            char name[64];
            snprintf(name, sizeof name, "  hsa pool %zu", i);
            time_writes(name, (unsigned*)p, (unsigned*)p);
        }
    }
    // reference: pinned host memory written by the CPU, read by the device over PCIe
    unsigned *h = nullptr, *hd = nullptr;
    hipHostMalloc((void**)&h, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void**)&hd, h, 0);
    time_writes("  pinned host", h, hd);
    return 0;
}
