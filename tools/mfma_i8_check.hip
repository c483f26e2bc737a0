// Exact-integer check of v_mfma_i32_16x16x64_i8 as flat_bf16_k64<I8> uses it: lane (m = l & 15, g = l >> 4) holds
// A[m][16g + j] and B[16g + j][n = m] in byte j of its 16-B fragment; C[4g + i][m] in accumulator i.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const signed char *A, const signed char *B, int *C) {
    const int l = threadIdx.x, m = l & 15, g = l >> 4;
    i32x4 a, b, c = {0, 0, 0, 0};
    signed char *pa = reinterpret_cast<signed char *>(&a), *pb = reinterpret_cast<signed char *>(&b);
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[m * 64 + 16 * g + j];
        pb[j] = B[(16 * g + j) * 16 + m];
    }
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + m] = c[i];
}
int main() {
    signed char hA[16 * 64], hB[64 * 16];
    int ref[256], out[256];
    for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)((i * 37 + 11) % 255 - 127);
    for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)((i * 53 + 7) % 251 - 125);
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            int s = 0;
            for (int kk = 0; kk < 64; ++kk) s += hA[r * 64 + kk] * hB[kk * 16 + c];
            ref[r * 16 + c] = s;
        }
    signed char *dA, *dB;
    int *dC;
    if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dC, sizeof out)) return 2;
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(out, dC, sizeof out, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += out[i] != ref[i];
    std::printf("mfma_i32_16x16x64_i8 map check: %d of 256 wrong (C[0][0] %d ref %d)\n", bad, out[0], ref[0]);
    return bad ? 1 : 0;
}
