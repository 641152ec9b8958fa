// hostreg_probe — how this ROCm reports page-locked host ranges (round 6):
// hipHostGetFlags vs hipPointerGetAttributes on a hipHostRegister range, its interior
// and last byte, double registration and unregistration. Log: profiles/r06_hostreg_probe.log
// Build: hipcc -O1 --offload-arch=gfx950 -o ab/hostreg_probe tools/hostreg_probe.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
static void q(const char* what, void* p) {
  unsigned f = 0;
  hipError_t a = hipHostGetFlags(&f, p);
  (void)hipGetLastError();
  hipPointerAttribute_t at{};
  hipError_t b = hipPointerGetAttributes(&at, p);
  (void)hipGetLastError();
  printf("%-28s getflags=%d(%u) ptrattr=%d type=%d hostPointer=%p devicePointer=%p\n", what, (int)a, f, (int)b,
         (int)at.type, at.hostPointer, at.devicePointer);
}
int main() {
  const size_t n = 64 << 20;
  char* m = (char*)aligned_alloc(4096, n);
  for (size_t i = 0; i < n; i += 4096) m[i] = 1;
  q("pageable", m);
  hipError_t r = hipHostRegister(m, n / 2, hipHostRegisterDefault);
  printf("register(first half) = %d\n", (int)r);
  q("registered base", m);
  q("registered interior", m + 12345);
  q("registered last byte", m + n / 2 - 1);
  q("past the range", m + n / 2 + 100);
  r = hipHostRegister(m, n / 2, hipHostRegisterDefault);
  printf("register again = %d\n", (int)r); (void)hipGetLastError();
  r = hipHostRegister(m + 4096, 4096, hipHostRegisterDefault);
  printf("register inner = %d\n", (int)r); (void)hipGetLastError();
  r = hipHostUnregister(m);
  printf("unregister = %d\n", (int)r); (void)hipGetLastError();
  q("after unregister", m);
  r = hipHostUnregister(m);
  printf("unregister again = %d\n", (int)r); (void)hipGetLastError();
  void* h = nullptr;
  hipHostMalloc(&h, 4096, 0);
  q("hipHostMalloc", h);
  return 0;
}
