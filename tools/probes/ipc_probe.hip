// Probe: which allocation kinds / sizes can be exported with hipIpcGetMemHandle.
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
  size_t sizes[] = {16384, 655360, 2u << 20, 4u << 20};
  unsigned flags[] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault};
  const char* names[] = {"uncached", "finegrained", "default"};
  for (int f = 0; f < 3; ++f)
    for (size_t s : sizes) {
      void* p = nullptr;
      hipError_t e = hipExtMallocWithFlags(&p, s, flags[f]);
      hipIpcMemHandle_t h;
      hipError_t e2 = e == hipSuccess ? hipIpcGetMemHandle(&h, p) : e;
      printf("%-12s %8zu alloc=%s ipc=%s\n", names[f], s, hipGetErrorString(e), hipGetErrorString(e2));
    }
  for (size_t s : sizes) {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, s);
    hipIpcMemHandle_t h;
    hipError_t e2 = hipIpcGetMemHandle(&h, p);
    printf("%-12s %8zu alloc=%s ipc=%s\n", "hipMalloc", s, hipGetErrorString(e), hipGetErrorString(e2));
  }
  return 0;
}
