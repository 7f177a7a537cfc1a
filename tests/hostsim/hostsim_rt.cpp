// Host-simulation runtime (see hip/hip_runtime.h). TEST INFRASTRUCTURE ONLY.
#include "hip/hip_runtime.h"

#include <atomic>
#include <mutex>
#include <string>

thread_local dim3 threadIdx;
thread_local dim3 blockIdx;
dim3 blockDim;
dim3 gridDim;
std::barrier<>* pk_sim_barrier = nullptr;

// Kernels that never call __syncthreads run without barriers: a few workers take whole blocks
// and run their threads one after another.
static void launch_independent(dim3 grid, dim3 block, const std::function<void()>& body) {
    gridDim = grid;
    blockDim = block;
    const unsigned nw = 8;
    std::vector<std::thread> ts;
    for (unsigned w = 0; w < nw; w++)
        ts.emplace_back([&, w]() {
            for (unsigned b = w; b < grid.x; b += nw) {
                blockIdx = dim3(b);
                for (unsigned t = 0; t < block.x; t++) {
                    threadIdx = dim3(t);
                    body();
                }
            }
        });
    for (auto& th : ts) th.join();
}

void pk_sim_launch(const char* name, dim3 grid, dim3 block, const std::function<void()>& body) {
    // the only kernel with __shared__ + __syncthreads (pk_step.hip launches it as PK_K1_KERNEL)
    while (*name == '(') name++;
    if (strncmp(name, "pk_step_kernel", 14) != 0 && strncmp(name, "PK_K1_KERNEL", 12) != 0) {
        launch_independent(grid, block, body);
        return;
    }
    // blockDim.x OS threads walk the blocks in order; a barrier at the end of every block keeps
    // the per-block __shared__ statics private to the block being run.
    gridDim = grid;
    blockDim = block;
    std::barrier<> bar((ptrdiff_t)block.x);
    pk_sim_barrier = &bar;
    std::vector<std::thread> ts;
    ts.reserve(block.x);
    for (unsigned t = 0; t < block.x; t++)
        ts.emplace_back([&, t]() {
            for (unsigned b = 0; b < grid.x; b++) {
                blockIdx = dim3(b);
                threadIdx = dim3(t);
                body();
                bar.arrive_and_wait();
            }
        });
    for (auto& th : ts) th.join();
}

#include <atomic>
#include <mutex>
static std::vector<uint32_t> g_trace;
static uint32_t g_trace_env = 0xFFFFFFFFu;
static size_t g_trace_cap = 0;
static std::mutex g_trace_mu;
extern "C" void pk_sim_trace_enable(uint32_t env, uint64_t cap) {
    std::lock_guard<std::mutex> l(g_trace_mu);
    g_trace.clear();
    g_trace_env = env;
    g_trace_cap = cap;
}
extern "C" void pk_sim_trace(uint32_t env, uint32_t pc, uint32_t w0, uint32_t w1, uint32_t sp, uint32_t op) {
    if (env != g_trace_env) return;
    std::lock_guard<std::mutex> l(g_trace_mu);
    if (g_trace.size() / 6 >= g_trace_cap) return;
    uint32_t rec[6] = {pc, w0, w1, sp, op, 0};
    g_trace.insert(g_trace.end(), rec, rec + 6);
}
extern "C" uint64_t pk_sim_trace_get(uint32_t* out, uint64_t cap) {
    std::lock_guard<std::mutex> l(g_trace_mu);
    uint64_t n = g_trace.size() / 6;
    if (n > cap) n = cap;
    memcpy(out, g_trace.data(), n * 6 * 4);
    return n;
}

// ---- per-iteration event recording (PK_ITER) ----
static std::vector<std::vector<uint32_t>> g_iter;
static std::vector<std::vector<uint32_t>> g_iter_op;
static bool g_iter_on = false;
extern "C" void pk_sim_iter_enable(uint32_t n_envs, int on) {
    g_iter.assign(on ? n_envs : 0, {});
    g_iter_op.assign(on ? n_envs : 0, {});
    g_iter_on = on != 0;
}
extern "C" void pk_sim_iter(uint32_t env, uint32_t ev) {
    if (!g_iter_on || env >= g_iter.size()) return;
    g_iter[env].push_back(ev);   // one env is stepped by one thread: no lock needed
}
extern "C" void pk_sim_iter_op(uint32_t env, uint32_t di) {
    if (!g_iter_on || env >= g_iter_op.size()) return;
    g_iter_op[env].push_back(di);
}
// fast-path RAM-image accesses: per env, (iteration << 20) | (kind << 16) | phys (iteration = the
// env's PK_ITER count so far, so accesses of one wave iteration can be grouped)
static std::vector<std::vector<uint64_t>> g_mem;
static bool g_mem_on = false;
extern "C" void pk_sim_mem_enable(uint32_t n_envs, int on) {
    g_mem.assign(on ? n_envs : 0, {});
    g_mem_on = on != 0;
}
extern "C" void pk_sim_memref(uint32_t env, uint32_t kind, uint32_t phys) {
    if (!g_mem_on || env >= g_mem.size()) return;
    const uint64_t it = env < g_iter.size() ? g_iter[env].size() : 0;
    g_mem[env].push_back((it << 20) | ((uint64_t)(kind & 3u) << 16) | (phys & 0xFFFFu));
}
extern "C" uint64_t pk_sim_mem_get(uint32_t env, uint64_t* out, uint64_t cap) {
    if (env >= g_mem.size()) return 0;
    uint64_t n = g_mem[env].size();
    if (out) memcpy(out, g_mem[env].data(), (n < cap ? n : cap) * 8);
    return n;
}
extern "C" uint64_t pk_sim_iter_op_get(uint32_t env, uint32_t* out, uint64_t cap) {
    if (env >= g_iter_op.size()) return 0;
    uint64_t n = g_iter_op[env].size();
    if (out) memcpy(out, g_iter_op[env].data(), (n < cap ? n : cap) * 4);
    return n;
}
extern "C" uint64_t pk_sim_iter_get(uint32_t env, uint32_t* out, uint64_t cap) {
    if (env >= g_iter.size()) return 0;
    uint64_t n = g_iter[env].size();
    if (out) memcpy(out, g_iter[env].data(), (n < cap ? n : cap) * 4);
    return n;
}

// ---- K1 lane-invariant failures (PK_CHECK, pk_step.hip pk_check_lane) ----
static std::mutex g_check_mu;
static uint64_t g_check_n = 0;
static std::string g_check_first, g_check_msg;
extern "C" void pk_sim_check_fail(uint32_t env, const char* what) {
    std::lock_guard<std::mutex> l(g_check_mu);
    if (g_check_n++ == 0) g_check_first = "K1 invariant: " + std::string(what) + " (env " + std::to_string(env) + ")";
}
// reported (and cleared) once: the first failure's text and the count
extern "C" int pk_sim_check_pending(void) {
    std::lock_guard<std::mutex> l(g_check_mu);
    if (!g_check_n) return 0;
    g_check_msg = g_check_first + ", " + std::to_string(g_check_n) + " failed checks";
    g_check_n = 0;
    return 1;
}
extern "C" const char* pk_sim_check_message(void) { return g_check_msg.c_str(); }

// ---- flush_lines statistics (PK_FLUSH_STAT): calls, lines rasterised ----
static std::atomic<uint64_t> g_flush_calls{0}, g_flush_lines{0};
extern "C" void pk_sim_flush_stat(uint32_t rendered) { (rendered ? g_flush_lines : g_flush_calls)++; }
extern "C" void pk_sim_flush_get(uint64_t* out) { out[0] = g_flush_calls.exchange(0); out[1] = g_flush_lines.exchange(0); }
