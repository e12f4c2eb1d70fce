// Kernel-boundary cost vs in-kernel grid barrier cost on MI355X.
//  A: back-to-back empty kernels (stream), B: same as a hipGraph, C: kernels that each write 1 MB,
//  D: one persistent kernel doing many grid barriers (agent-scope release/acquire + arrival counter),
//     optionally writing 4 KB per workgroup between barriers.
// Every spin loop is bounded (a failed barrier sets an error flag and exits), so the grid always drains.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_k(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}

__global__ void write_k(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = i; j < n; j += gridDim.x * blockDim.x) p[j] = (float)j;
}

__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned nblocks, unsigned& gen, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned target = (gen + 1) * nblocks;
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1L << 24)) {
        ok = false;
        atomicExch(err, 1);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  ++gen;
  __syncthreads();
  return ok && !__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void persist_k(unsigned* bar, int iters, float* buf, int write, int* err) {
  unsigned gen = 0;
  for (int it = 0; it < iters; ++it) {
    if (write) {
      float* my = buf + (long)blockIdx.x * 1024;
      // read the neighbour's slice written before the previous barrier, write mine
      const float* nb = buf + (long)((blockIdx.x + 37) % gridDim.x) * 1024;
      float v = nb[(threadIdx.x * 4) & 1023];
      for (int j = threadIdx.x; j < 1024; j += 256) my[j] = v + j + it;
    }
    if (!grid_barrier(bar, gridDim.x, gen, err)) return;
  }
}

template <class F>
static float timeit(F f, hipStream_t st) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipStreamSynchronize(st);
  hipEventRecord(a, st);
  f();
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  const int NK = 2000;
  float* buf;
  hipMalloc(&buf, 64 << 20);
  unsigned* bar;
  int* err;
  hipMalloc(&bar, 4096);
  hipMalloc(&err, 4096);
  for (int g : {1, 256, 2048}) {
    float ms = timeit([&] {
      for (int i = 0; i < NK; ++i) hipLaunchKernelGGL(empty_k, dim3(g), dim3(256), 0, st, nullptr);
    }, st);
    printf("A stream empty kernel grid=%5d: %6.2f us/kernel\n", g, ms * 1000 / NK);
  }
  for (int g : {1, 256, 2048}) {
    hipGraph_t graph;
    hipGraphExec_t exec;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < NK; ++i) hipLaunchKernelGGL(empty_k, dim3(g), dim3(256), 0, st, nullptr);
    hipStreamEndCapture(st, &graph);
    hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    float ms = timeit([&] { hipGraphLaunch(exec, st); }, st);
    printf("B graph  empty kernel grid=%5d: %6.2f us/kernel\n", g, ms * 1000 / NK);
    hipGraphExecDestroy(exec);
    hipGraphDestroy(graph);
  }
  for (int n : {1 << 18, 1 << 20}) {
    float ms = timeit([&] {
      for (int i = 0; i < NK; ++i) hipLaunchKernelGGL(write_k, dim3(256), dim3(256), 0, st, buf, n);
    }, st);
    printf("C stream write %7d B kernel: %6.2f us/kernel\n", n * 4, ms * 1000 / NK);
  }
  for (int g : {256, 512, 1024}) {
    for (int w : {0, 1}) {
      hipMemset(bar, 0, 4096);
      hipMemset(err, 0, 4096);
      hipDeviceSynchronize();
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a, st);
      hipLaunchKernelGGL(persist_k, dim3(g), dim3(256), 0, st, bar, NK, buf, w, err);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      int e;
      hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
      printf("D persistent grid=%4d write=%d: %6.2f us/barrier  err=%d\n", g, w, ms * 1000 / NK, e);
    }
  }
  return 0;
}
