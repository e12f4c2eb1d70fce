// Two decode chains on one GPU: how HIP runs the parallel branches of ONE captured graph, and what a cross-branch
// edge costs, against the two-streams-two-graphs form the decode uses today.
//   A  one chain of N spin kernels, one stream, one graph                       (the reference time of one chain)
//   B  two chains as the two branches of one graph (fork / join by events)      (parallel -> ~A, serial -> ~2A)
//   C  B plus a cross edge every `e` kernels: chain-2 kernel i waits for chain-1 kernel i (a pinned offset)
//   D  two graphs (one chain each) launched on two streams by one host thread
// Spin kernels hold their workgroups for a fixed device-clock time (s_memrealtime, 100 MHz), so the numbers are
// scheduling cost, not memory behaviour. Every spin is bounded by its own tick count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void spin_k(unsigned long long ticks, int* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (sink && threadIdx.x == 0 && (t & 0xffffffffffffULL) == 1) sink[blockIdx.x] = 1;  // never true in practice
}

static void chain(hipStream_t st, int n, unsigned long long ticks, int grid) {
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(spin_k, dim3(grid), dim3(64), 0, st, ticks, nullptr);
}

static float time_graph(hipGraphExec_t g, hipStream_t st, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraphLaunch(g, st);
  hipStreamSynchronize(st);
  hipEventRecord(a, st);
  for (int r = 0; r < reps; ++r) hipGraphLaunch(g, st);
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

int main() {
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int N = 64, reps = 20, grid = 80;
  for (double us : {2.0, 5.0, 20.0}) {
    const unsigned long long ticks = (unsigned long long)(us * 100.0);
    // A
    hipGraph_t gA;
    hipGraphExec_t xA;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    chain(s1, N, ticks, grid);
    CK(hipStreamEndCapture(s1, &gA));
    CK(hipGraphInstantiate(&xA, gA, nullptr, nullptr, 0));
    const float a = time_graph(xA, s1, reps);
    // D: two graphs, two streams, one host thread
    hipGraphExec_t xA2;
    CK(hipGraphInstantiate(&xA2, gA, nullptr, nullptr, 0));
    float d = 0;
    {
      hipEvent_t e0, e1, f2;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventCreate(&f2);
      hipGraphLaunch(xA, s1);
      hipGraphLaunch(xA2, s2);
      hipDeviceSynchronize();
      hipEventRecord(e0, s1);
      hipStreamWaitEvent(s2, e0, 0);
      for (int r = 0; r < reps; ++r) {
        hipGraphLaunch(xA, s1);
        hipGraphLaunch(xA2, s2);
      }
      hipEventRecord(f2, s2);
      hipStreamWaitEvent(s1, f2, 0);
      hipEventRecord(e1, s1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&d, e0, e1);
      d /= reps;
    }
    printf("spin %5.1f us x %d kernels, %d WGs: A one chain %8.1f us (%6.2f us/kernel) | D two graphs two streams "
           "%8.1f us (%.2fx A)\n", us, N, grid, a * 1000, a * 1000 / N, d * 1000, d / a);
    // B / C: one graph, two branches, cross edges every e kernels (e = 0: none)
    for (int e : {0, 8, 4, 1}) {
      std::vector<hipEvent_t> ev(2 * N + 2);
      for (auto& x : ev) hipEventCreateWithFlags(&x, hipEventDisableTiming);
      hipGraph_t gB;
      hipGraphExec_t xB;
      CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
      hipEventRecord(ev[0], s1);
      hipStreamWaitEvent(s2, ev[0], 0);  // fork
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(spin_k, dim3(grid), dim3(64), 0, s1, ticks, nullptr);
        if (e > 0 && (i % e) == 0) {
          hipEventRecord(ev[2 + i], s1);
          hipStreamWaitEvent(s2, ev[2 + i], 0);  // chain-2 kernel i starts after chain-1 kernel i
        }
        hipLaunchKernelGGL(spin_k, dim3(grid), dim3(64), 0, s2, ticks, nullptr);
      }
      hipEventRecord(ev[1], s2);
      hipStreamWaitEvent(s1, ev[1], 0);  // join
      CK(hipStreamEndCapture(s1, &gB));
      size_t nn = 0;
      hipGraphGetNodes(gB, nullptr, &nn);
      CK(hipGraphInstantiate(&xB, gB, nullptr, nullptr, 0));
      const float b = time_graph(xB, s1, reps);
      printf("   one graph, two branches, cross edge every %d: %8.1f us (%.2fx A; %zu nodes)\n", e, b * 1000, b / a, nn);
      hipGraphExecDestroy(xB);
      hipGraphDestroy(gB);
      for (auto& x : ev) hipEventDestroy(x);
    }
    hipGraphExecDestroy(xA);
    hipGraphExecDestroy(xA2);
    hipGraphDestroy(gA);
  }
  return 0;
}
