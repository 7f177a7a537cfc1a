// Host-simulation shim for the HIP runtime — TEST INFRASTRUCTURE ONLY.
//
// Lets tests compile the unmodified kernels (pokegym_amd/csrc/pk_kernels.hip) and C ABI
// (pk_capi.cpp) with g++ and run them on the CPU: every workgroup runs as blockDim OS threads
// joined by a std::barrier at __syncthreads(); __shared__ arrays are per-block statics (one block
// runs at a time).  Device memory is host memory.  This checks kernel LOGIC against the oracle
// without a GPU; the real gfx950 build is what ships and is checked by the -m gpu tests.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <barrier>
#include <functional>
#include <thread>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __shared__ static
#define __constant__ static const
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
#define __builtin_amdgcn_readfirstlane(x) (x)
#define __builtin_amdgcn_s_setprio(x) ((void)0)
#define __builtin_amdgcn_s_waitcnt(x) ((void)0)
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
#define PK_PIN3(a, b, c) ((void)0)
#define PK_OPAQUE(x) ((void)0)
// lanes run one at a time: a ballot of this lane alone (uses test ballot(x) != 0 for "any lane")
#define __builtin_amdgcn_ballot_w64(x) ((uint64_t)(bool)(x))
// v_perm_b32: byte i of the result = byte sel.byte[i] of {hi, lo} (0-3 lo, 4-7 hi), 8-11 the sign
// bit of lo[15], lo[31], hi[15], hi[31] replicated, 0x0C -> 0x00, >= 0x0D -> 0xFF
static inline uint32_t __builtin_amdgcn_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t s = (sel >> (8 * i)) & 0xFFu, b;
        if (s < 8) b = (uint32_t)(v >> (8 * s)) & 0xFFu;
        else if (s == 0x0C) b = 0;
        else if (s > 0x0C) b = 0xFF;
        else {  // 8..11: replicate the sign bit of lo[15], lo[31], hi[15], hi[31]
            static const int bitpos[4] = {15, 31, 47, 63};
            b = ((v >> bitpos[s - 8]) & 1u) ? 0xFFu : 0u;
        }
        r |= b << (8 * i);
    }
    return r;
}
// v_bfe_u32: width bits at offset (both & 31); width 0 -> 0
static inline uint32_t __builtin_amdgcn_ubfe(uint32_t src, uint32_t off, uint32_t width) {
    off &= 31u;
    width &= 31u;
    if (width == 0u) return 0u;
    if (off + width >= 32u) return src >> off;
    return (src << (32u - off - width)) >> (32u - width);
}
// v_bfe_i32: width bits at offset (both & 31), sign-extended; width 0 -> 0
static inline int __builtin_amdgcn_sbfe(int src, uint32_t off, uint32_t width) {
    off &= 31u;
    width &= 31u;
    if (width == 0u) return 0;
    if (off + width >= 32u) return (int)src >> off;
    return (int)((uint32_t)src << (32u - off - width)) >> (32u - width);
}
// v_alignbyte_b32: ({hi, lo} >> (8 * (sh & 3)))[31:0]
static inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (sh & 3)));
}
using std::max;
using std::min;

struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct uint2 { uint32_t x, y; };
struct uint4 { uint32_t x, y, z, w; };
static inline uint2 make_uint2(uint32_t a, uint32_t b) { return uint2{a, b}; }
static inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }

extern thread_local dim3 threadIdx;
extern thread_local dim3 blockIdx;
extern dim3 blockDim;
extern dim3 gridDim;
extern std::barrier<>* pk_sim_barrier;
static inline void __syncthreads() { pk_sim_barrier->arrive_and_wait(); }

typedef int hipError_t;
typedef void* hipStream_t;
typedef void* hipEvent_t;
enum { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2 };
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice, hipMemcpyHostToHost };
// K1's lane-invariant checks (pk_step.hip pk_check_lane): a failed check is recorded
// (hostsim_rt.cpp) and reported by the next hipGetLastError — the launch's own error check in
// pk_launch_step — so the C ABI call that ran the kernel fails with the first failure's text
enum { hipErrorAssert = 710 };
extern "C" int pk_sim_check_pending(void);
extern "C" const char* pk_sim_check_message(void);
static inline const char* hipGetErrorString(hipError_t e) { return e == hipErrorAssert ? pk_sim_check_message() : "hostsim error"; }
static inline hipError_t hipGetLastError() { return pk_sim_check_pending() ? (hipError_t)hipErrorAssert : hipSuccess; }
extern "C" void pk_sim_check_fail(uint32_t env, const char* what);
#ifndef PK_NO_CHECK
#define PK_CHECK(env, cond, what) do { if (!(cond)) pk_sim_check_fail(env, what); } while (0)
#endif
static inline hipError_t hipSetDevice(int) { return hipSuccess; }
static inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 1 };
static inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = 256; return hipSuccess; }
static inline hipError_t hipMalloc(void** p, size_t n) {
    *p = aligned_alloc(256, (n + 255) / 256 * 256);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
static inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
static inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { memmove(d, s, n); return hipSuccess; }
static inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) { memmove(d, s, n); return hipSuccess; }
static inline hipError_t hipMemset(void* d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
static inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
static inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
static inline hipError_t hipEventCreate(hipEvent_t* e) { *e = nullptr; return hipSuccess; }
static inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
static inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
static inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
static inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }

void pk_sim_launch(const char* name, dim3 grid, dim3 block, const std::function<void()>& body);
#define hipLaunchKernelGGL(k, grid, block, shmem, stream, ...) \
    pk_sim_launch(#k, dim3(grid), dim3(block), [&]() { k(__VA_ARGS__); })

// instruction trace for debugging (env, pc, w0, w1, sp, opcode)
extern "C" void pk_sim_trace(uint32_t env, uint32_t pc, uint32_t w0, uint32_t w1, uint32_t sp, uint32_t op);
#define PK_TRACE(env, pc, w0, w1, sp, op) pk_sim_trace(env, pc, w0, w1, sp, op)
// loop fast-path marker: op = 0x1000 | loop length, w0 = passes run (tools/trace_diff.py)
#define PK_TRACE_SKIP(env, pc, passes, len) pk_sim_trace(env, pc, passes, 0u, 0u, 0x1000u | (len))

// per-iteration event bits (iteration statistics for kernel design; see pk_kernels.hip PK_EV_*)
extern "C" void pk_sim_iter(uint32_t env, uint32_t ev);
#define PK_ITER(env, ev) pk_sim_iter(env, ev)
// per-iteration microcode index (design statistics: opcode uniformity of a wave)
extern "C" void pk_sim_iter_op(uint32_t env, uint32_t di);
#define PK_ITER_OP(env, di) pk_sim_iter_op(env, di)
// flush_lines calls (0) and the lines they rasterise (1) (design statistics)
extern "C" void pk_sim_flush_stat(uint32_t rendered);
#define PK_FLUSH_STAT(rendered) pk_sim_flush_stat(rendered)
// fast-path RAM-image accesses (tools/mem_stats.py)
extern "C" void pk_sim_memref(uint32_t env, uint32_t kind, uint32_t phys);
#define PK_MEMREF(env, kind, phys) pk_sim_memref(env, kind, phys)
