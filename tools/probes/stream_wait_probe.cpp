// Probe: which memory kinds support hipStreamWaitValue64 (CP wait) + hipStreamWriteValue64 across streams,
// and which can be exported through HIP IPC. Every wait is bounded (host polls hipStreamQuery for 3 s).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

static const char* name(hipError_t e) { return hipGetErrorString(e); }

static void probe(const char* label, uint64_t* p) {
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  hipError_t e1 = hipStreamWaitValue64(a, p, 5, hipStreamWaitValueGte);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  hipError_t q0 = hipStreamQuery(a);  // expected: not ready (still waiting)
  hipError_t e2 = hipStreamWriteValue64(b, p, 7, 0);
  hipStreamSynchronize(b);
  bool done = false;
  for (int i = 0; i < 300 && !done; ++i) {
    done = hipStreamQuery(a) == hipSuccess;
    if (!done) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  hipIpcMemHandle_t h;
  hipError_t e3 = hipIpcGetMemHandle(&h, p);
  printf("%-28s wait=%s before_write=%s write=%s completed=%d ipc_export=%s\n", label, name(e1), name(q0), name(e2),
         (int)done, name(e3));
  fflush(stdout);
  if (!done) {  // unblock the waiter before leaving
    hipStreamWriteValue64(b, p, 100, 0);
    hipStreamSynchronize(b);
  }
}

int main() {
  hipSetDevice(0);
  int attr = 0;
  hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("CanUseStreamWaitValue=%d\n", attr);
  uint64_t* d = nullptr;
  hipMalloc(&d, 4096);
  hipMemset(d, 0, 4096);
  hipDeviceSynchronize();
  probe("hipMalloc", d);
  uint64_t* s8 = nullptr;
  hipError_t es = hipExtMallocWithFlags((void**)&s8, 8, hipMallocSignalMemory);
  printf("signal alloc(8): %s\n", name(es));
  if (es == hipSuccess) { hipMemset(s8, 0, 8); hipDeviceSynchronize(); probe("signal(8)", s8); }
  uint64_t* fg = nullptr;
  hipError_t ef = hipExtMallocWithFlags((void**)&fg, 4096, hipDeviceMallocFinegrained);
  printf("finegrained alloc: %s\n", name(ef));
  if (ef == hipSuccess) { hipMemset(fg, 0, 4096); hipDeviceSynchronize(); probe("finegrained", fg); }
  uint64_t* uc = nullptr;
  hipError_t eu = hipExtMallocWithFlags((void**)&uc, 4096, hipDeviceMallocUncached);
  printf("uncached alloc: %s\n", name(eu));
  if (eu == hipSuccess) { hipMemset(uc, 0, 4096); hipDeviceSynchronize(); probe("uncached", uc); }
  uint64_t* hm = nullptr;
  hipHostMalloc((void**)&hm, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hm[0] = 0;
  probe("hostmalloc coherent", hm);
  return 0;
}
