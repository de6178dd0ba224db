// FETCH_SIZE calibration for the access shapes the flat decides use
// (MI355X_MICROARCH.md: the x2 correction is measured for 16-B/lane streaming
// reads only; "calibrate on a known byte count in your own access pattern").
// Three kernels over a 2 GiB buffer (past the 256 MiB Infinity Cache), each
// reading a known set of lines once:
//   k_stream   16 B per lane, coalesced: 2 GiB
//   k_hdr24    one thread per 1 KiB record: 24 B at the record start (six
//              dwords, the FlatHdr read) -> one 64-B half-line / one 128-B line per record
//   k_edge16   one thread per 1 KiB record: 16 B at offset 512 (an edge chunk)
//   k_halves   one thread per 1 KiB record: 4 B at offsets 0 and 64 (both halves of a line)
// rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib prints the per-dispatch KiB;
// scripts/gpu_fetch_calib.sh compares them with these byte counts.
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib scripts/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void k_stream(const uint4* __restrict__ p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads
}
__global__ void k_hdr24(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t* sink) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint32_t* w = (const uint32_t*)(p + r * 1024);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) acc ^= w[k];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void k_edge16(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t* sink) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint4 v = *(const uint4*)(p + r * 1024 + 512);
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// both 64-B halves of one 128-B line per record (4 B at offsets 0 and 64):
// one request per record if the L2 fetches 128-B lines, two if 64-B sectors
__global__ void k_halves(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t* sink) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint32_t acc = *(const uint32_t*)(p + r * 1024) ^ *(const uint32_t*)(p + r * 1024 + 64);
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
  const uint64_t bytes = 2ull << 30, nrec = bytes / 1024;
  uint8_t* p = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  (void)hipMemset(p, 1, bytes);
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)p, bytes / 16, sink);
    hipLaunchKernelGGL(k_hdr24, dim3((uint32_t)((nrec + 255) / 256)), dim3(256), 0, 0, p, nrec, sink);
    hipLaunchKernelGGL(k_edge16, dim3((uint32_t)((nrec + 255) / 256)), dim3(256), 0, 0, p, nrec, sink);
    hipLaunchKernelGGL(k_halves, dim3((uint32_t)((nrec + 255) / 256)), dim3(256), 0, 0, p, nrec, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes %llu records %llu: k_stream reads %llu B; k_hdr24 / k_edge16 touch %llu lines of 128 B (%llu B)\n",
         (unsigned long long)bytes, (unsigned long long)nrec, (unsigned long long)bytes, (unsigned long long)nrec,
         (unsigned long long)(nrec * 128));
  (void)hipFree(p);
  (void)hipFree(sink);
  return 0;
}
