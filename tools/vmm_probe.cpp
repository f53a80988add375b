// HBM arenas through HIP's virtual memory management API, for tools/vmm_probe.py (tuning probe, not shipped).
//
// The encode / decode rate follows the allocation a buffer lands in (profiles/r03/placement/), and no
// virtual-address offset or contiguity request predicted it.  One candidate is how the GPU page tables map
// the buffer: a reservation aligned to a large power of two, backed by physical handles of a large
// granularity, lets the driver use large translation fragments.  vmm_alloc reserves `size` bytes of virtual
// address space aligned to `va_align`, backs it with physical handles of `chunk` bytes (0 = one handle),
// maps them in order and grants the device read/write access.
//
// build: hipcc -O2 -shared -fPIC tools/vmm_probe.cpp -o tools/libvmm_probe.so
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

namespace {
struct Arena {
    size_t size;
    std::vector<hipMemGenericAllocationHandle_t> handles;
};
std::map<void*, Arena> g_arenas;

hipMemAllocationProp prop_for(int dev) {
    hipMemAllocationProp p = {};
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}
}  // namespace

extern "C" int vmm_granularity(size_t* minimum, size_t* recommended) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipMemAllocationProp p = prop_for(dev);
    if (hipMemGetAllocationGranularity(minimum, &p, hipMemAllocationGranularityMinimum) != hipSuccess) return -2;
    if (hipMemGetAllocationGranularity(recommended, &p, hipMemAllocationGranularityRecommended) != hipSuccess) return -3;
    return 0;
}

extern "C" void* vmm_alloc(size_t size, size_t va_align, size_t chunk) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    hipMemAllocationProp p = prop_for(dev);
    if (chunk == 0) chunk = size;
    if (size % chunk != 0) return nullptr;
    void* base = nullptr;
    hipError_t e = hipMemAddressReserve(&base, size, va_align, nullptr, 0);
    if (e != hipSuccess) {
        fprintf(stderr, "hipMemAddressReserve: %s\n", hipGetErrorString(e));
        return nullptr;
    }
    Arena a{size, {}};
    for (size_t off = 0; off < size; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        e = hipMemCreate(&h, chunk, &p, 0);
        if (e == hipSuccess) {
            a.handles.push_back(h);
            e = hipMemMap((char*)base + off, chunk, 0, h, 0);
        }
        if (e != hipSuccess) {
            fprintf(stderr, "hipMemCreate/Map at %zu: %s\n", off, hipGetErrorString(e));
            for (size_t i = 0; i < a.handles.size(); i++) {
                if (i * chunk < off) (void)hipMemUnmap((char*)base + i * chunk, chunk);
                (void)hipMemRelease(a.handles[i]);
            }
            (void)hipMemAddressFree(base, size);
            return nullptr;
        }
    }
    hipMemAccessDesc d = {};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = dev;
    d.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(base, size, &d, 1);
    if (e != hipSuccess) {
        fprintf(stderr, "hipMemSetAccess: %s\n", hipGetErrorString(e));
        return nullptr;
    }
    g_arenas[base] = a;
    return base;
}

extern "C" int vmm_free(void* base) {
    auto it = g_arenas.find(base);
    if (it == g_arenas.end()) return -1;
    const size_t chunk = it->second.size / it->second.handles.size();
    for (size_t i = 0; i < it->second.handles.size(); i++) {
        (void)hipMemUnmap((char*)base + i * chunk, chunk);
        (void)hipMemRelease(it->second.handles[i]);
    }
    (void)hipMemAddressFree(base, it->second.size);
    g_arenas.erase(it);
    return 0;
}
