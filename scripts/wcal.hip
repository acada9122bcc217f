// Write-counter calibration (the fed engine's write accounting): kernels that each write a known number
// of bytes with one of the store forms the resident engine uses, so rocprofv3's WRITE_SIZE per dispatch can be read
// as bytes-per-store for that form (MI355X_MICROARCH.md: WRITE_SIZE is exact only for 16-byte-per-lane streaming
// stores; calibrate every other width on a known count). Run: rocprofv3 --pmc WRITE_SIZE -- scripts/build/wcal
// (scripts/write_account.sh). Each kernel prints nothing; the host prints the byte and store counts per kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kT = 256;
constexpr size_t kN = 1 << 20;  // lanes of the coalesced kernels

// plain coalesced stores: 4 B (the sweepers' keys), 8 B (their static cache), 16 B (the reference form)
__global__ void w_plain4(uint32_t* p) { p[blockIdx.x * kT + threadIdx.x] = threadIdx.x; }
__global__ void w_plain8(uint64_t* p) { p[blockIdx.x * kT + threadIdx.x] = threadIdx.x; }
__global__ void w_plain16(uint4* p) { p[blockIdx.x * kT + threadIdx.x] = make_uint4(1, 2, 3, threadIdx.x); }
// relaxed agent-scope atomic stores (the engine's st_sc1 / x_store64 / tag_store): coalesced 8 B (the selector's
// entry words, published sets), coalesced 4 B (commit lists), and one 8-B word per 128-B line (row columns of scattered
// nodes, single tagged words)
__global__ void w_at8(uint64_t* p) {
  __hip_atomic_store(&p[blockIdx.x * kT + threadIdx.x], (uint64_t)threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void w_at4(uint32_t* p) {
  __hip_atomic_store(&p[blockIdx.x * kT + threadIdx.x], (uint32_t)threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void w_at8_scatter(uint64_t* p) {
  __hip_atomic_store(&p[(size_t)(blockIdx.x * kT + threadIdx.x) * 16], (uint64_t)threadIdx.x, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// the level records: eight 4-B stores per lane at a 32-B record stride
__global__ void w_plain4_rec(uint32_t* p) {
  uint32_t* o = p + (size_t)(blockIdx.x * kT + threadIdx.x) * 8;
#pragma unroll 1
  for (int j = 0; j < 8; ++j) o[j] = (uint32_t)j;
}
// plain 8-B coalesced stores followed by an agent-scope release per wave (the sweepers' per-job release)
__global__ void w_plain8_release(uint64_t* p) {
  p[blockIdx.x * kT + threadIdx.x] = threadIdx.x;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

int main() {
  void* buf = nullptr;
  const size_t bytes = kN * 16 * 16;  // room for the scattered form
  if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipDeviceSynchronize();
  const dim3 g(kN / kT), b(kT), gs(kN / 16 / kT), gr(kN / 8 / kT);
  for (int rep = 0; rep < 3; ++rep) {  // (repeated: the first dispatch of each may pay first-touch)
    hipLaunchKernelGGL(w_plain4, g, b, 0, 0, (uint32_t*)buf);
    hipLaunchKernelGGL(w_plain8, g, b, 0, 0, (uint64_t*)buf);
    hipLaunchKernelGGL(w_plain16, g, b, 0, 0, (uint4*)buf);
    hipLaunchKernelGGL(w_at8, g, b, 0, 0, (uint64_t*)buf);
    hipLaunchKernelGGL(w_at4, g, b, 0, 0, (uint32_t*)buf);
    hipLaunchKernelGGL(w_at8_scatter, gs, b, 0, 0, (uint64_t*)buf);
    hipLaunchKernelGGL(w_plain4_rec, gr, b, 0, 0, (uint32_t*)buf);
    hipLaunchKernelGGL(w_plain8_release, g, b, 0, 0, (uint64_t*)buf);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  // bytes written and store instructions (lanes) per dispatch
  printf("{\"w_plain4\": [%zu, %zu], \"w_plain8\": [%zu, %zu], \"w_plain16\": [%zu, %zu], \"w_at8\": [%zu, %zu], "
         "\"w_at4\": [%zu, %zu], \"w_at8_scatter\": [%zu, %zu], \"w_plain4_rec\": [%zu, %zu], "
         "\"w_plain8_release\": [%zu, %zu]}\n",
         kN * 4, kN, kN * 8, kN, kN * 16, kN, kN * 8, kN, kN * 4, kN, kN / 16 * 8, kN / 16, kN / 8 * 32, kN / 8,
         kN * 8, kN);
  hipFree(buf);
  return 0;
}
