// VMM behaviour probe: reserve, map two chunks back to back, set access per
// chunk / on the whole range; a kernel writes and reads both.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); printf("%-60s -> %s\n", #x, hipGetErrorString(e)); } while (0)

__global__ void touch(unsigned* p, size_t n, unsigned* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = (unsigned)i;
  __syncthreads();
  if (i < n && p[i] != (unsigned)i) atomicAdd(out, 1u);
}

int main() {
  int dev = 0, vmm = 0;
  hipSetDevice(dev);
  CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev));
  printf("vmm=%d\n", vmm);
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gmin = 0, grec = 0;
  CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  printf("gran min=%zu rec=%zu\n", gmin, grec);
  size_t g = grec, R = 64 * g;
  void* base = nullptr;
  CK(hipMemAddressReserve(&base, R, g, nullptr, 0));
  hipMemGenericAllocationHandle_t h1, h2, h3;
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemCreate(&h1, 2 * g, &prop, 0));
  CK(hipMemMap(base, 2 * g, 0, h1, 0));
  CK(hipMemSetAccess(base, 2 * g, &acc, 1));
  char* b = (char*)base;
  CK(hipMemCreate(&h2, 3 * g, &prop, 0));
  CK(hipMemMap(b + 2 * g, 3 * g, 0, h2, 0));
  printf("-- access on the second chunk only\n");
  CK(hipMemSetAccess(b + 2 * g, 3 * g, &acc, 1));
  (void)hipGetLastError();
  printf("-- access on the whole mapped range\n");
  CK(hipMemSetAccess(base, 5 * g, &acc, 1));
  (void)hipGetLastError();
  CK(hipMemCreate(&h3, 1 * g, &prop, 0));
  CK(hipMemMap(b + 5 * g, g, 0, h3, 0));
  printf("-- third chunk: access on the chunk\n");
  CK(hipMemSetAccess(b + 5 * g, g, &acc, 1));
  (void)hipGetLastError();
  printf("-- third chunk: access on whole\n");
  CK(hipMemSetAccess(base, 6 * g, &acc, 1));
  (void)hipGetLastError();
  unsigned* out;
  hipMalloc(&out, 4);
  hipMemset(out, 0, 4);
  size_t n = 6 * g / 4;
  hipLaunchKernelGGL(touch, dim3((n + 255) / 256), dim3(256), 0, 0, (unsigned*)base, n, out);
  CK(hipDeviceSynchronize());
  unsigned bad = 0;
  hipMemcpy(&bad, out, 4, hipMemcpyDeviceToHost);
  printf("bad=%u\n", bad);
  CK(hipMemsetAsync(b + 2 * g, 0, g, 0));
  CK(hipDeviceSynchronize());
  CK(hipMemUnmap(base, 2 * g));
  CK(hipMemUnmap(b + 2 * g, 3 * g));
  CK(hipMemUnmap(b + 5 * g, g));
  CK(hipMemRelease(h1));
  CK(hipMemRelease(h2));
  CK(hipMemRelease(h3));
  CK(hipMemAddressFree(base, R));
  return 0;
}
