// Does a freed uncached allocation's address come back from plain hipMalloc?
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
    hipSetDevice(0);
    for (size_t sz : {(size_t)1 << 20, (size_t)1 << 21, (size_t)3 << 20, (size_t)64 << 20}) {
        void *uc = nullptr, *a = nullptr, *b = nullptr;
        hipExtMallocWithFlags(&uc, sz, hipDeviceMallocUncached);
        hipFree(uc);
        hipMalloc(&a, sz);
        hipMalloc(&b, sz);
        printf("size %zu: uncached %p -> hipMalloc %p %p  reuse=%d\n", sz, uc, a, b, (a == uc) || (b == uc));
        hipFree(a); hipFree(b);
    }
    return 0;
}
