// Microbenchmark: what a chain of small dependent kernels costs per launch on one
// stream, launched one by one vs replayed as an instantiated HIP graph, and with
// host syncs in the middle (the online per-call path: ~32 launches and 2 host
// round trips per RunConsensus).  Each kernel is one 64-thread
// block that bumps a counter (no work: the cost is dispatch and completion).
//   launch_gap [launches per call] [calls]
// prints microseconds per call for: stream launches + 1 sync, the same as a graph,
// stream launches with 2 syncs (half and half), the graph split at the sync, and
// a graph re-captured per call (new arguments) and updated in place before its launch.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_tiny(int* p) {
  if (threadIdx.x == 0) p[0] += 1;
}

// the engine's kernels take a ~300-byte Tables struct by value
struct Big {
  int* p;
  int v[72];
};
__global__ void k_big(Big b) {
  if (threadIdx.x == 0) b.p[0] += b.v[threadIdx.x & 63];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the same struct read through a device pointer (8 bytes of arguments)
__global__ void k_bigp(const Big* __restrict__ b) {
  if (threadIdx.x == 0) b->p[0] += b->v[threadIdx.x & 63];
}

// `launch_gap args L C`: argument size alone, interleaved A/B (8-byte pointer to a
// device copy of the struct vs the 292-byte struct by value), 6 alternations
static int args_ab(int L, int C) {
  int* d;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Big bg;
  bg.p = d;
  for (int i = 0; i < 72; i++) bg.v[i] = i;
  Big* db;
  CK(hipMalloc(&db, sizeof(Big)));
  CK(hipMemcpy(db, &bg, sizeof(Big), hipMemcpyHostToDevice));
  auto run = [&](int kind) {
    const double t0 = now_us();
    for (int c = 0; c < C; c++) {
      for (int i = 0; i < L; i++) {
        if (kind) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, bg);
        else hipLaunchKernelGGL(k_bigp, dim3(1), dim3(64), 0, st, (const Big*)db);
      }
      CK(hipStreamSynchronize(st));
    }
    return (now_us() - t0) / C;
  };
  run(0);
  run(1);
  printf("{\"launches_per_call\": %d, \"calls\": %d, \"arg_bytes\": [8, %zu], \"ptr_us\": [", L, C, sizeof(Big));
  double v[2][6];
  for (int r = 0; r < 6; r++) {
    v[0][r] = run(0);
    v[1][r] = run(1);
  }
  for (int r = 0; r < 6; r++) printf("%s%.1f", r ? ", " : "", v[0][r]);
  printf("], \"byvalue_us\": [");
  for (int r = 0; r < 6; r++) printf("%s%.1f", r ? ", " : "", v[1][r]);
  printf("]}\n");
  return 0;
}

// `launch_gap copies L C`: what small stream-ordered copies cost inside a chain of
// L launches (the online call's control uploads and result downloads): per call,
// L launches + 1 sync with 0, 2 or 4 small copies (1 KB H2D from pinned memory,
// then 1 KB D2H into pinned memory), vs the same data read and written by the
// kernels themselves straight from / to pinned host memory (no copy operations)
__global__ void k_zc(const int* __restrict__ hin, int* __restrict__ hout, int* d) {
  if (threadIdx.x < 64) {
    const int v = hin[threadIdx.x];
    if (threadIdx.x == 0) d[0] += v;
    hout[threadIdx.x] = v + 1;
  }
}
static int copies_ab(int L, int C) {
  int *d, *dbuf, *hp, *hq;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  CK(hipMalloc(&dbuf, 4096));
  CK(hipHostMalloc((void**)&hp, 4096, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hq, 4096, hipHostMallocDefault));
  for (int i = 0; i < 1024; i++) hp[i] = i;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto run = [&](int ncopy, bool zc) {
    const double t0 = now_us();
    for (int c = 0; c < C; c++) {
      for (int i = 0; i < L; i++) {
        if (ncopy && i == 0) CK(hipMemcpyAsync(dbuf, hp, 1024, hipMemcpyHostToDevice, st));
        if (ncopy > 2 && i == L / 2) {
          CK(hipMemcpyAsync(hq, dbuf, 1024, hipMemcpyDeviceToHost, st));
          CK(hipMemcpyAsync(dbuf, hp, 1024, hipMemcpyHostToDevice, st));
        }
        if (zc && (i == 0 || i == L / 2 || i == L - 1)) hipLaunchKernelGGL(k_zc, dim3(1), dim3(64), 0, st, hp, hq, d);
        else hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, d);
      }
      if (ncopy) CK(hipMemcpyAsync(hq, dbuf, 1024, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
    }
    return (now_us() - t0) / C;
  };
  run(0, false);
  run(4, false);
  run(0, true);
  double v[4][5];
  for (int r = 0; r < 5; r++) {
    v[0][r] = run(0, false);
    v[1][r] = run(2, false);
    v[2][r] = run(4, false);
    v[3][r] = run(0, true);
  }
  const char* nm[4] = {"no_copies_us", "copies2_us", "copies4_us", "zero_copy_us"};
  printf("{\"launches_per_call\": %d, \"calls\": %d", L, C);
  for (int k = 0; k < 4; k++) {
    printf(", \"%s\": [", nm[k]);
    for (int r = 0; r < 5; r++) printf("%s%.1f", r ? ", " : "", v[k][r]);
    printf("]");
  }
  printf("}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'c') return copies_ab(argc > 2 ? atoi(argv[2]) : 16, argc > 3 ? atoi(argv[3]) : 2000);
  if (argc > 1 && argv[1][0] == 'a') return args_ab(argc > 2 ? atoi(argv[2]) : 20, argc > 3 ? atoi(argv[3]) : 2000);
  const int L = argc > 1 ? atoi(argv[1]) : 32, C = argc > 2 ? atoi(argv[2]) : 2000;
  int* d;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto launches = [&](int n) {
    for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, d);
  };
  // graphs: all L launches, and the two halves
  hipGraph_t g[3];
  hipGraphExec_t ge[3];
  const int parts[3] = {L, L / 2, L - L / 2};
  for (int k = 0; k < 3; k++) {
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    launches(parts[k]);
    CK(hipStreamEndCapture(st, &g[k]));
    CK(hipGraphInstantiate(&ge[k], g[k], nullptr, nullptr, 0));
  }
  for (int w = 0; w < 200; w++) {  // warm up (clocks, code objects)
    launches(L);
    CK(hipStreamSynchronize(st));
    CK(hipGraphLaunch(ge[0], st));
    CK(hipStreamSynchronize(st));
  }
  double t0 = now_us();
  for (int c = 0; c < C; c++) {
    launches(L);
    CK(hipStreamSynchronize(st));
  }
  const double a = (now_us() - t0) / C;
  t0 = now_us();
  for (int c = 0; c < C; c++) {
    CK(hipGraphLaunch(ge[0], st));
    CK(hipStreamSynchronize(st));
  }
  const double b = (now_us() - t0) / C;
  t0 = now_us();
  for (int c = 0; c < C; c++) {
    launches(L / 2);
    CK(hipStreamSynchronize(st));
    launches(L - L / 2);
    CK(hipStreamSynchronize(st));
  }
  const double a2 = (now_us() - t0) / C;
  t0 = now_us();
  for (int c = 0; c < C; c++) {
    CK(hipGraphLaunch(ge[1], st));
    CK(hipStreamSynchronize(st));
    CK(hipGraphLaunch(ge[2], st));
    CK(hipStreamSynchronize(st));
  }
  const double b2 = (now_us() - t0) / C;
  // per call: capture the launches (arguments differ per call, as the engine's do),
  // update the instantiated graph in place, launch it (what a per-call graph costs)
  hipGraphExec_t gu;
  {
    hipGraph_t g0;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    launches(L);
    CK(hipStreamEndCapture(st, &g0));
    CK(hipGraphInstantiate(&gu, g0, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g0));
  }
  int upd_fail = 0;
  double cap_us = 0, upd_us = 0;
  t0 = now_us();
  for (int c = 0; c < C; c++) {
    const double a0 = now_us();
    hipGraph_t gc;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < L; i++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, d + ((c + i) & 7));
    CK(hipStreamEndCapture(st, &gc));
    const double a1 = now_us();
    hipGraphExecUpdateResult r;
    hipGraphNode_t en;
    if (hipGraphExecUpdate(gu, gc, &en, &r) != hipSuccess) upd_fail++;
    const double a2 = now_us();
    CK(hipGraphLaunch(gu, st));
    CK(hipStreamSynchronize(st));
    CK(hipGraphDestroy(gc));
    cap_us += a1 - a0;
    upd_us += a2 - a1;
  }
  const double cu = (now_us() - t0) / C;
  Big bg;
  bg.p = d;
  for (int i = 0; i < 72; i++) bg.v[i] = i;
  t0 = now_us();
  for (int c = 0; c < C; c++) {
    for (int i = 0; i < L; i++) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, bg);
    CK(hipStreamSynchronize(st));
  }
  const double ab = (now_us() - t0) / C;
  t0 = now_us();
  for (int c = 0; c < C; c++) CK(hipStreamSynchronize(st));
  const double s = (now_us() - t0) / C;
  printf("{\"launches_per_call\": %d, \"calls\": %d, \"stream_1sync_us\": %.1f, \"graph_1sync_us\": %.1f, "
         "\"stream_2sync_us\": %.1f, \"graph_2sync_us\": %.1f, \"empty_sync_us\": %.2f, "
         "\"capture_update_launch_us\": %.1f, \"capture_us\": %.1f, \"update_us\": %.1f, \"update_failures\": %d, \"stream_1sync_300B_args_us\": %.1f}\n",
         L, C, a, b, a2, b2, s, cu, cap_us / C, upd_us / C, upd_fail, ab);
  return 0;
}
