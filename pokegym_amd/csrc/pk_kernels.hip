// pk_kernels.hip — MI355X (gfx950) kernels around the step kernel (K1 lives in pk_step.hip):
//
//   K2 pk_render_kernel  rasterises the scanlines latched during the last (rendered) frame into
//                        the persistent 144x160 u8 grey screen (replaces PyBoy's renderer +
//                        screen.screen_ndarray(), pokegym/environment.py:268).
//   K5 pk_reset_*        per-env copy of the parsed template savestate (pyboy_binding.py:66-69).
//   gather/scatter       one env's RAM image <-> a dense buffer (pk_snapshot / pk_load_env / peeks).
//   pk_done_kernel       termination flags when the reward stack is off (environment.py:1612-1613).
//
// Everything here is integer byte work; no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pk_layout.h"
#include "pk_render.h"

// ---------------------------------------------------------------------------------------------
// K2: rasterise the latched lines of the rendered frame.  One wave = one (group, scanline),
// lane = env: the 64 lanes read the same VRAM offsets of their interleaved images (coalesced).
__global__ void __launch_bounds__(64) pk_render_kernel(PkStepArgs A) {
    const u32 y = blockIdx.x % PK_ROWS;
    const u32 gid = A.env0 / PK_LANES + blockIdx.x / PK_ROWS;
    const u32 lane = threadIdx.x;
    const u32 env = gid * PK_LANES + lane;
    if (env >= A.env1) return;
    const u32 rf = A.regs[PK_R_RFLAGS * A.npad + env];
    u8* out = A.screen + (size_t)env * PK_SCREEN + y * PK_COLS;
    const u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
    const u32 l2 = A.lat[2u * A.lat_stride + idx];
    if (rf & 1u) {  // frame ended with the LCD off: blank_screen() (white); its latched lines are dropped
        uint4 wv;
        wv.x = wv.y = wv.z = wv.w = 0xFFFFFFFFu;
        for (u32 q = 0; q < PK_COLS; q += 16) *reinterpret_cast<uint4*>(out + q) = wv;
        if (l2 & 0x100u) A.lat[2u * A.lat_stride + idx] = l2 & ~0x100u;
        return;
    }
    if (!(l2 & 0x100u)) return;
    const Mem m = mem_view(A.mem, env, A.ilv_sh);
    render_line(m, y, A.lat[idx], A.lat[A.lat_stride + idx], (int)(l2 & 0xFFu) - 1, out);
    A.lat[2u * A.lat_stride + idx] = l2 & ~0x100u;
}

// Re-arm every env's 144 latched lines for K2 (pk_render_latched): the window line counter of each
// line follows from the latched LCDC/WY/WX as K1 derives it at latch time (pyboy renderer: the
// window counter advances on lines where the window is enabled, started and on screen).
__global__ void __launch_bounds__(256) pk_arm_latches_kernel(PkStepArgs A) {
    const u32 env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= A.n) return;
    const u32 gid = env / PK_LANES, lane = env % PK_LANES;
    int lw = -1;
    for (u32 y = 0; y < PK_ROWS; y++) {
        const u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
        const u32 l0 = A.lat[idx], l1 = A.lat[A.lat_stride + idx];
        const u32 wy = l1 & 0xFFu, wx = bfe8(l0, 24);
        if ((l0 & 0x20u) && wy <= y && (int)wx - 7 < (int)PK_COLS) lw += 1;
        A.lat[2u * A.lat_stride + idx] = (u32)(lw + 1) | 0x100u;
    }
    A.regs[PK_R_RFLAGS * A.npad + env] &= ~1u;
}

// ---------------------------------------------------------------------------------------------
// K5: reset selected envs from the template (regs + RAM image + screen + line latches).


// The reset kernels work on a device-built list of the envs to reset (pk_list_kernel: ids of the
// masked envs, count in device memory), so a step where few or no envs finish costs a few
// near-empty launches instead of a scan of every env's 49.7 KB image — and no host sync.
__global__ void __launch_bounds__(256) pk_list_kernel(const u8* mask, u32 env0, u32 env1, u32* cnt, u32* ids) {
    const u32 e = env0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= env1 || (mask && !mask[e])) return;
    ids[atomicAdd(cnt, 1u)] = e;
}

// template RAM image -> listed envs: thread = env (list order, so a wave's stores to one image
// row land in one 64-byte line when its envs share a group), block = a strided set of rows
__global__ void __launch_bounds__(256) pk_reset_mem_kernel(PkResetArgs A) {
    const u32 cnt = *A.cnt;
    for (u32 k = threadIdx.x; k < cnt; k += blockDim.x) {
        const u32 env = A.ids[k];
        const Mem m = mem_view(A.mem, env, A.ilv_sh);
        for (u32 p = blockIdx.x; p < PK_PHYS; p += gridDim.x) st_phys(m, p, A.tmpl_mem[p]);
    }
}

__global__ void __launch_bounds__(256) pk_reset_regs_kernel(PkResetArgs A) {
    const u32 cnt = *A.cnt;
    for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += gridDim.x * blockDim.x) {
        const u32 env = A.ids[k];
        for (u32 f = 0; f < PK_NREGS; f++) A.regs[f * A.npad + env] = A.tmpl_regs[f];
        const u32 gid = env / PK_LANES, lane = env % PK_LANES;
        for (u32 j = 0; j < 3u; j++)
            for (u32 y = 0; y < PK_ROWS; y++)
                A.lat[j * A.lat_stride + (gid * PK_ROWS + y) * PK_LANES + lane] = A.tmpl_lat[j * PK_ROWS + y];
        const uint4* s = reinterpret_cast<const uint4*>(A.tmpl_screen);
        uint4* d = reinterpret_cast<uint4*>(A.screen + (size_t)env * PK_SCREEN);
        for (u32 q = 0; q < PK_SCREEN / 16u; q++) d[q] = s[q];
    }
}

// gather one env's RAM image into a compact buffer (for pk_snapshot / pk_peek)
__global__ void pk_gather_env_kernel(const u8* mem, u32 env, u32 sh, u8* out) {
    const Mem m = mem_view(const_cast<u8*>(mem), env, sh);
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < PK_PHYS; p += gridDim.x * blockDim.x)
        out[p] = ld_phys(m, p);
}

// gather envs [env0, env0 + count) into out[count][PK_PHYS] (bulk snapshots): one thread per
// (phys row, env) with env fastest, so each wave reads consecutive interleaved bytes
__global__ void __launch_bounds__(256) pk_gather_range_kernel(const u8* mem, u32 env0, u32 count, u32 sh, u8* out) {
    const size_t total = (size_t)count * PK_PHYS;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const u32 k = (u32)(t % count), p = (u32)(t / count);
        const u32 env = env0 + k;
        out[(size_t)k * PK_PHYS + p] = mem[pk_img_off(env, p, sh)];
    }
}

__global__ void pk_scatter_env_kernel(u8* mem, u32 env, u32 sh, const u8* in) {
    const Mem m = mem_view(mem, env, sh);
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < PK_PHYS; p += gridDim.x * blockDim.x)
        st_phys(m, p, in[p]);
}

// ---------------------------------------------------------------------------------------------
// host-side launchers (called by the C ABI in pk_capi.cpp)
hipError_t pk_launch_render(const PkStepArgs& a, hipStream_t s) {
    const u32 grid = ((a.env1 - a.env0 + PK_LANES - 1u) / PK_LANES) * PK_ROWS;
    hipLaunchKernelGGL(pk_render_kernel, dim3(grid), dim3(PK_LANES), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_render_latched(const PkStepArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_arm_latches_kernel, dim3((a.env1 + 255) / 256), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return pk_launch_render(a, s);
}

hipError_t pk_launch_list(const u8* mask, u32 env0, u32 env1, u32* cnt, u32* ids, hipStream_t s) {
    hipLaunchKernelGGL(pk_list_kernel, dim3((env1 - env0 + 255) / 256), dim3(256), 0, s, mask, env0, env1, cnt, ids);
    return hipGetLastError();
}

// reset the envs listed in (a.cnt, a.ids)
hipError_t pk_launch_reset(const PkResetArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_reset_mem_kernel, dim3(4096), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pk_reset_regs_kernel, dim3((a.env1 - a.env0 + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_gather_env(const u8* mem, u32 env, u32 sh, u8* out, hipStream_t s) {
    hipLaunchKernelGGL(pk_gather_env_kernel, dim3(64), dim3(256), 0, s, mem, env, sh, out);
    return hipGetLastError();
}

hipError_t pk_launch_gather_range(const u8* mem, u32 env0, u32 count, u32 sh, u8* out, hipStream_t s) {
    hipLaunchKernelGGL(pk_gather_range_kernel, dim3(2048), dim3(256), 0, s, mem, env0, count, sh, out);
    return hipGetLastError();
}

hipError_t pk_launch_scatter_env(u8* mem, u32 env, u32 sh, const u8* in, hipStream_t s) {
    hipLaunchKernelGGL(pk_scatter_env_kernel, dim3(64), dim3(256), 0, s, mem, env, sh, in);
    return hipGetLastError();
}

__global__ void pk_done_kernel(const u32* time_reg, u32 n, u32 max_steps, u8* term, u8* trunc, double* rew) {
    const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const u8 done = time_reg[e] >= max_steps ? 1 : 0;
    if (term) term[e] = done;
    if (trunc) trunc[e] = done;
    if (rew) rew[e] = 0.0;
}

hipError_t pk_launch_done(const u32* time_reg, u32 n, u32 max_steps, u8* term, u8* trunc, double* rew, hipStream_t s) {
    hipLaunchKernelGGL(pk_done_kernel, dim3((n + 255) / 256), dim3(256), 0, s, time_reg, n, max_steps, term, trunc, rew);
    return hipGetLastError();
}
