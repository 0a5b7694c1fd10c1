// Microbenchmark: the cost of cross-stream event ordering between two HIP streams of one device, in
// the pattern of the pipelined env step (capi.hip msc_env_step): a long "demand" kernel on a side
// stream, a chain of shorter "step" kernels on the main stream, each waiting on the other's event.
// Build: hipcc --offload-arch=gfx950 -O2 tools/ev_gap.hip -o tools/ev_gap
// Prints the per-iteration period of each pattern next to the spin length of its kernels.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// every wave spins for `ticks` of the 100 MHz real-time counter, then one lane per block stores
__global__ void spin(unsigned long long ticks, unsigned* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)t0;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  const unsigned long long dem = 75000, stp = 60000;  // 750 us, 600 us (100 MHz)
  const unsigned flags_list[3] = {hipEventDisableTiming, hipEventDisableTiming | hipEventReleaseToDevice,
                                  hipEventDisableTiming | hipEventDisableSystemFence};
  const char* fname[3] = {"default", "device", "nofence"};
  unsigned* out;
  CK(hipMalloc(&out, 4096 * sizeof(unsigned)));
  hipStream_t main_s, side;
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  const int blocks = 512;
  // stream memory operations instead of events (patterns 6, 7): one 32-bit counter per direction
  unsigned *cnt_dem = nullptr, *cnt_step = nullptr;
  CK(hipExtMallocWithFlags((void**)&cnt_dem, 8, hipMallocSignalMemory));
  CK(hipExtMallocWithFlags((void**)&cnt_step, 8, hipMallocSignalMemory));
  for (int f = 0; f < 3; f++) {
    hipEvent_t ev_dem[2], ev_step[2];
    for (int b = 0; b < 2; b++) {
      CK(hipEventCreateWithFlags(&ev_dem[b], flags_list[f]));
      CK(hipEventCreateWithFlags(&ev_step[b], flags_list[f]));
      CK(hipEventRecord(ev_dem[b], side));
      CK(hipEventRecord(ev_step[b], side));
    }
    hipEvent_t ev_pre;
    CK(hipEventCreateWithFlags(&ev_pre, flags_list[f]));
    CK(hipEventRecord(ev_pre, main_s));
    CK(hipDeviceSynchronize());
    for (int pat = 0; pat < 8; pat++) {
      // 0: demand kernels back to back on one stream
      // 1: the same with an event record after each
      // 2: the pipelined pattern (side: wait step(t-1), demand(t+1), record; main: wait demand(t), 3 step kernels, record)
      // 3: pattern 2 with the demand on the main stream's side swapped (step chain longer than demand)
      // 4: pattern 2 without the side stream's wait (main waits on the demand only)
      // 5: demand kernels, each after a wait on an event completed long before
      // 6: pattern 2 with hipStreamWriteValue32 / hipStreamWaitValue32 (>=) on counters instead of events
      // 7: pattern 6 without the side stream's wait
      for (int rep = 0; rep < 2; rep++) {
        CK(hipDeviceSynchronize());
        const double t0 = now_ms();
        for (int t = 0; t < iters; t++) {
          const int b = t & 1;
          if (pat == 0) {
            spin<<<blocks, 64, 0, side>>>(dem, out);
          } else if (pat == 1) {
            spin<<<blocks, 64, 0, side>>>(dem, out);
            CK(hipEventRecord(ev_dem[b], side));
          } else if (pat >= 6) {
            if (t == 0) {
              CK(hipMemsetAsync(cnt_dem, 0, 8, side));
              CK(hipMemsetAsync(cnt_step, 0, 8, side));
              CK(hipStreamSynchronize(side));
            }
            // demand t is signalled as count t + 1 (demand 0 is "done" before the loop)
            CK(hipStreamWaitValue32(main_s, cnt_dem, (unsigned)t, hipStreamWaitValueGte, 0xffffffffu));
            spin<<<blocks, 64, 0, main_s>>>(stp / 30, out + 1024);
            spin<<<blocks, 64, 0, main_s>>>(stp * 20 / 30, out + 2048);
            spin<<<blocks, 64, 0, main_s>>>(stp * 9 / 30, out + 3072);
            CK(hipStreamWriteValue32(main_s, cnt_step, (unsigned)t + 1, 0));
            if (pat == 6 && t >= 1) CK(hipStreamWaitValue32(side, cnt_step, (unsigned)t, hipStreamWaitValueGte, 0xffffffffu));
            spin<<<blocks, 64, 0, side>>>(dem, out);
            CK(hipStreamWriteValue32(side, cnt_dem, (unsigned)t + 1, 0));
          } else if (pat == 5) {
            CK(hipStreamWaitEvent(side, ev_pre, 0));
            spin<<<blocks, 64, 0, side>>>(dem, out);
          } else {
            const unsigned long long d = pat == 3 ? stp : dem, s = pat == 3 ? dem : stp;
            CK(hipStreamWaitEvent(main_s, ev_dem[b], 0));
            spin<<<blocks, 64, 0, main_s>>>(s / 30, out + 1024);
            spin<<<blocks, 64, 0, main_s>>>(s * 20 / 30, out + 2048);
            spin<<<blocks, 64, 0, main_s>>>(s * 9 / 30, out + 3072);
            CK(hipEventRecord(ev_step[b], main_s));
            if (pat != 4)
              CK(hipStreamWaitEvent(side, ev_step[b ^ 1], 0));
            spin<<<blocks, 64, 0, side>>>(d, out);
            CK(hipEventRecord(ev_dem[b ^ 1], side));
          }
        }
        CK(hipDeviceSynchronize());
        const double ms = (now_ms() - t0) / iters;
        if (rep == 1)
          printf("flags=%-8s pattern=%d period=%.4f ms (demand spin %.3f ms, step spin %.3f ms)\n", fname[f], pat, ms,
                 dem / 1e5, stp / 1e5);
      }
    }
    CK(hipEventDestroy(ev_pre));
    for (int b = 0; b < 2; b++) {
      CK(hipEventDestroy(ev_dem[b]));
      CK(hipEventDestroy(ev_step[b]));
    }
  }
  CK(hipFree(out));
  CK(hipFree(cnt_dem));
  CK(hipFree(cnt_step));
  return 0;
}
