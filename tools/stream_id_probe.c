#include <hip/hip_runtime_api.h>
#include <stdio.h>
int main(void) {
  unsigned long long id0 = 0;
  hipError_t e0 = hipStreamGetId((hipStream_t)0, &id0);
  printf("{\"null\": {\"rc\": %d, \"id\": %llu}, \"rows\": [", (int)e0, id0);
  for (int i = 0; i < 6; ++i) {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    unsigned long long id = 0;
    hipError_t e = hipStreamGetId(s, &id);
    printf("%s{\"ptr\": \"%p\", \"rc\": %d, \"id\": %llu}", i ? ", " : "", (void*)s, (int)e, id);
    if (hipStreamDestroy(s) != hipSuccess) return 2;
  }
  printf("]}\n");
  return 0;
}
