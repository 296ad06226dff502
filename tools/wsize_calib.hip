// WRITE_SIZE calibration for the store patterns of the Pacman turn rollout
// (MI355X_MICROARCH.md: "WRITE_SIZE reads the bytes exactly for 16-B-per-lane
// streaming stores ... other access widths are uncalibrated").  Three kernels
// write a KNOWN number of bytes; rocprofv3 --pmc WRITE_SIZE per dispatch over
// the byte count is the counter's factor for that pattern:
//   k_wide   16 B per lane, contiguous (the guide's calibrated case)
//   k_rows   pac_observe's pattern: one wave per env writes one 441-dword row
//            (21x21 int32) of its env's [5][441] block per turn, dword l + 64 k
//            per lane, nontemporal; 16384 envs x 10 turns
//   k_rows16 the same rows written with 16 B per lane where aligned (head and
//            tail dwords by single-dword stores)
// build: hipcc --offload-arch=gfx950 -O3 -o wsize_calib tools/wsize_calib.hip
// run:   rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR -o run -- ./wsize_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int E = 16384, A = 5, HW = 441, TURNS = 10;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void k_wide(i32x4* out, size_t n16)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const i32x4 v = {1, 2, 3, (int)i};
    if (i < n16) __builtin_nontemporal_store(v, out + i);
}

__global__ void k_rows(int32_t* obs)
{
    const int e = blockIdx.x, l = threadIdx.x;
    for (int t = 0; t < TURNS; t++) {
        const int a = (e + t) % A;
        int32_t* out = obs + (((size_t)t * E + e) * A + a) * HW;
        for (int i = l; i < HW; i += 64) __builtin_nontemporal_store(i ^ e, out + i);
    }
}

__global__ void k_rows16(int32_t* obs)
{
    const int e = blockIdx.x, l = threadIdx.x;
    for (int t = 0; t < TURNS; t++) {
        const int a = (e + t) % A;
        int32_t* out = obs + (((size_t)t * E + e) * A + a) * HW;
        const int head = (int)((4 - (((uintptr_t)out >> 2) & 3)) & 3);   // dwords before a 16-B boundary
        if (l < head) __builtin_nontemporal_store(l ^ e, out + l);
        const int n4 = (HW - head) / 4;
        i32x4* o4 = (i32x4*)(out + head);
        for (int i = l; i < n4; i += 64) {
            const i32x4 v = {i, e, 0, 1};
            __builtin_nontemporal_store(v, o4 + i);
        }
        const int tail = HW - head - 4 * n4;
        if (l < tail) __builtin_nontemporal_store(l ^ e, out + head + 4 * n4 + l);
    }
}

int main()
{
    const size_t rows_bytes = (size_t)TURNS * E * A * HW * 4;
    const size_t wide_bytes = (size_t)256 << 20;
    void *obs, *wide;
    if (hipMalloc(&obs, rows_bytes) != hipSuccess || hipMalloc(&wide, wide_bytes) != hipSuccess) return 1;
    if (hipMemset(obs, 0, rows_bytes) != hipSuccess || hipMemset(wide, 0, wide_bytes) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const size_t n16 = wide_bytes / 16;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_wide, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, (i32x4*)wide, n16);
        hipLaunchKernelGGL(k_rows, dim3(E), dim3(64), 0, 0, (int32_t*)obs);
        hipLaunchKernelGGL(k_rows16, dim3(E), dim3(64), 0, 0, (int32_t*)obs);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("k_wide bytes %zu\nk_rows bytes %zu\nk_rows16 bytes %zu\n", wide_bytes,
           (size_t)TURNS * E * HW * 4, (size_t)TURNS * E * HW * 4);
    return hipFree(obs) != hipSuccess || hipFree(wide) != hipSuccess;
}
