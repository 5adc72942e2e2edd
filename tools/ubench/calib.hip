// PMC calibration: stream-read a known number of bytes with the eval/solver
// access widths (4 B and 8 B per lane, coalesced) and write a known number
// of bytes with 8 B per lane, so that FETCH_SIZE / WRITE_SIZE per dispatch can
// be converted to bytes for this code's access pattern
// (MI355X_MICROARCH.md: widths other than 16 B/lane are uncalibrated).
// Buffers are 1 GiB each, far past the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void read_i32(const int32_t* __restrict__ a, int64_t n, int64_t* out) {
    int64_t s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 0x7fffffffffffLL) out[0] = s;
}
__global__ void read_f64(const double* __restrict__ a, int64_t n, double* out) {
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 1.2345) out[0] = s;
}
__global__ void write_f64(double* __restrict__ a, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

int main() {
    const int64_t bytes = 1LL << 30;
    void *a, *b, *o;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 64)) return 1;
    (void)hipMemset(a, 0, bytes);
    (void)hipMemset(b, 0, bytes);
    (void)hipDeviceSynchronize();
    for (int it = 0; it < 2; ++it) {
        read_i32<<<4096, 256>>>((const int32_t*)a, bytes / 4, (int64_t*)o);
        read_f64<<<4096, 256>>>((const double*)b, bytes / 8, (double*)o);
        write_f64<<<4096, 256>>>((double*)a, bytes / 8);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("calib: each kernel moves %lld bytes\n", (long long)bytes);
    return 0;
}
