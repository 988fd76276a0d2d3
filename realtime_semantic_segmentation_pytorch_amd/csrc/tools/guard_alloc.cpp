// Guard-page device allocator: a debugging stand-in for PyTorch's caching allocator
// (torch.cuda.memory.CUDAPluggableAllocator) that makes every out-of-bounds access of a
// kernel fault on the FIRST launch that does it, independent of allocation history.
//
// Every allocation gets its own virtual range  [guard | mapped pages | guard]  built with
// the HIP virtual-memory API (hipMemAddressReserve / hipMemCreate / hipMemMap); the guard
// granules are reserved but never mapped.  RTSEG_GUARD_MODE selects where the tensor sits:
//   tail (default): the tensor ends less than 256 bytes before the first guard byte (its
//                   start stays 256-byte aligned: libraries such as MIOpen assume that; the
//                   caching allocator leaves up to 511 bytes after a tensor at a segment end,
//                   so every overrun that can fault in production faults here);
//   head:           the tensor STARTS at the mapped base; any access before it faults.
// RTSEG_GUARD_FILL=zero|nan fills fresh memory with zeros or 0xFF bytes (a NaN in fp32 / bf16 /
// fp16): a kernel that consumes memory it never wrote then shows up as a NaN or a mismatch.
// Used by tests/test_guard_alloc_gpu.py and tools/gpu_r3_guard.sh to pin the round-2
// intermittent illegal-address fault (profiles/r3_fault/README.md).  Slow (one mapping per
// tensor, a device synchronisation per free): a test tool, never a training path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace {

struct Block {
  void* va;
  size_t reserved;
  size_t mapped;
  void* mapped_base;
  hipMemGenericAllocationHandle_t handle;
};

std::mutex g_mu;
std::unordered_map<void*, Block> g_blocks;
size_t g_gran = 0;
int g_tail = -1;
int g_fill = -1;  // byte value, or 256 = leave fresh memory as it comes
size_t g_live_bytes = 0, g_peak_bytes = 0, g_count = 0;

void die(const char* what, hipError_t e) {
  std::fprintf(stderr, "[rtseg_guard] %s failed: %s\n", what, hipGetErrorString(e));
  std::abort();
}

hipMemAllocationProp prop_for(int device) {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof(p));
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

}  // namespace

extern "C" {

void* rtseg_guard_malloc(ssize_t size, int device, hipStream_t) {
  if (size <= 0) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_tail < 0) {
    const char* m = std::getenv("RTSEG_GUARD_MODE");
    g_tail = (m && std::strcmp(m, "head") == 0) ? 0 : 1;
  }
  hipMemAllocationProp prop = prop_for(device);
  if (g_gran == 0) {
    hipError_t e = hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityMinimum);
    if (e != hipSuccess) die("hipMemGetAllocationGranularity", e);
  }
  const size_t need = (static_cast<size_t>(size) + 255) & ~static_cast<size_t>(255);
  const size_t mapped = (need + g_gran - 1) / g_gran * g_gran;
  const size_t reserved = mapped + 2 * g_gran;
  Block b{};
  b.reserved = reserved;
  b.mapped = mapped;
  hipError_t e = hipMemAddressReserve(&b.va, reserved, g_gran, nullptr, 0);
  if (e != hipSuccess) die("hipMemAddressReserve", e);
  e = hipMemCreate(&b.handle, mapped, &prop, 0);
  if (e != hipSuccess) die("hipMemCreate", e);
  b.mapped_base = static_cast<char*>(b.va) + g_gran;
  e = hipMemMap(b.mapped_base, mapped, 0, b.handle, 0);
  if (e != hipSuccess) die("hipMemMap", e);
  hipMemAccessDesc acc;
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = device;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  e = hipMemSetAccess(b.mapped_base, mapped, &acc, 1);
  if (e != hipSuccess) die("hipMemSetAccess", e);
  void* p = g_tail ? static_cast<char*>(b.mapped_base) + (mapped - need) : b.mapped_base;
  if (g_fill < 0) {
    const char* f = std::getenv("RTSEG_GUARD_FILL");
    g_fill = (f && std::strcmp(f, "nan") == 0) ? 0xFF : (f && std::strcmp(f, "zero") == 0) ? 0 : 256;
  }
  if (g_fill != 256) {
    e = hipMemset(b.mapped_base, g_fill, mapped);
    if (e != hipSuccess) die("hipMemset", e);
  }
  g_blocks[p] = b;
  g_live_bytes += mapped;
  if (g_live_bytes > g_peak_bytes) g_peak_bytes = g_live_bytes;
  ++g_count;
  return p;
}

void rtseg_guard_free(void* ptr, ssize_t, int, hipStream_t) {
  if (ptr == nullptr) return;
  // the tensor may still be in use by queued kernels: drain before unmapping
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) die("hipDeviceSynchronize (a kernel before this free faulted)", e);
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_blocks.find(ptr);
  if (it == g_blocks.end()) {
    std::fprintf(stderr, "[rtseg_guard] free of unknown pointer %p\n", ptr);
    std::abort();
  }
  Block b = it->second;
  g_blocks.erase(it);
  g_live_bytes -= b.mapped;
  if ((e = hipMemUnmap(b.mapped_base, b.mapped)) != hipSuccess) die("hipMemUnmap", e);
  if ((e = hipMemRelease(b.handle)) != hipSuccess) die("hipMemRelease", e);
  if ((e = hipMemAddressFree(b.va, b.reserved)) != hipSuccess) die("hipMemAddressFree", e);
}

// (allocations made, live mapped bytes, peak mapped bytes, granularity)
void rtseg_guard_stats(size_t* out4) {
  std::lock_guard<std::mutex> lk(g_mu);
  out4[0] = g_count;
  out4[1] = g_live_bytes;
  out4[2] = g_peak_bytes;
  out4[3] = g_gran;
}

}  // extern "C"
