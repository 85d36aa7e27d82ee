// ftar_kernels.hip -- CDNA4 (gfx950) kernels of the fault-tolerant Allreduce.
//
// Every kernel here is HBM- or xGMI-bound integer/float streaming work: one pass over
// the operands, no reuse, no MFMA.  What matters on MI355X:
//   * 16-byte lanes (global_load_dwordx4 / global_store_dwordx4): 1 KiB per wave
//     instruction, the widest coalesced access;
//   * enough bytes in flight and short-lived blocks: one 16 KiB tile per operand per
//     256-thread workgroup, four independent 16-byte non-temporal loads per lane and
//     operand, non-temporal stores, one tile per block (32768 workgroups for the 256 MiB
//     C2 reduce) -- the fastest mapping of the rotating-buffer sweep (tools/hbm_sweep.hip);
//   * one launch handles up to FDEV_MAX_KSEGS independent segments (e.g. Raben's
//     step 0: reduce half the window + copy the other half of the partner's vector),
//     blocks are split between segments in proportion to their bytes and each wave
//     finds its segment with a wave-uniform (readfirstlane) search;
//   * segments whose pointers are not co-aligned to 16 bytes are split by the host
//     into a scalar head, a vector body and a scalar tail.
// Peer (xGMI) pointers obtained through hipIpcOpenMemHandle are plain device pointers
// here: the same kernel is the local reduce and the fused "pull + reduce" exchange.
//
// Reference semantics restated: MPI_Reduce_local(in, inout) = inout <op> in with
// OpenMPI's operand roles (out = out + in; max: out = (out > in) ? out : in), see
// include/ftar.h.  int32/int64 SUM/PROD wrap (two's complement), floats are one IEEE
// op per element (-ffp-contract=off, no fast-math).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <type_traits>

#include "ftar_kernels.h"

namespace ftar {

// ---------------------------------------------------------------------------------
// element ops
// ---------------------------------------------------------------------------------
template <typename T> struct Arith { using U = T; };
template <> struct Arith<int32_t> { using U = uint32_t; };
template <> struct Arith<int64_t> { using U = uint64_t; };

template <typename T, int OP>
__device__ __forceinline__ T apply(T x, T y)
{
    using U = typename Arith<T>::U;
    if constexpr (OP == kSum) return (T)((U)x + (U)y);
    else if constexpr (OP == kProd) return (T)((U)x * (U)y);
    else if constexpr (OP == kMax) return (x > y) ? x : y;
    else if constexpr (OP == kMin) return (x < y) ? x : y;
    // MPI's logical and bitwise ops (integer types only; the logical ones give 0 / 1)
    else if constexpr (OP == kLand) return (T)((x != 0) && (y != 0));
    else if constexpr (OP == kBand) return (T)(x & y);
    else if constexpr (OP == kLor) return (T)((x != 0) || (y != 0));
    else if constexpr (OP == kBor) return (T)(x | y);
    else if constexpr (OP == kLxor) return (T)((x != 0) != (y != 0));
    else return (T)(x ^ y);
}

// Runs fn(std::integral_constant<int, OP>) for the runtime op: one instantiation per op
// the element type has (the logical / bitwise ops only for the integer types).
template <typename T, typename Fn>
static hipError_t with_op(int op, Fn &&fn)
{
    using std::integral_constant;
    constexpr bool integer = std::is_integral<T>::value;
    switch (op) {
    case kSum: return fn(integral_constant<int, kSum>{});
    case kProd: return fn(integral_constant<int, kProd>{});
    case kMax: return fn(integral_constant<int, kMax>{});
    case kMin: return fn(integral_constant<int, kMin>{});
    default: break;
    }
    if constexpr (integer) {
        switch (op) {
        case kLand: return fn(integral_constant<int, kLand>{});
        case kBand: return fn(integral_constant<int, kBand>{});
        case kLor: return fn(integral_constant<int, kLor>{});
        case kBor: return fn(integral_constant<int, kBor>{});
        case kLxor: return fn(integral_constant<int, kLxor>{});
        case kBxor: return fn(integral_constant<int, kBxor>{});
        default: break;
        }
    }
    return hipErrorInvalidValue;
}

template <typename T, int OP>
__device__ __forceinline__ uint4 apply16(uint4 a, uint4 b)
{
    constexpr int E = 16 / sizeof(T);
    T xa[E], xb[E];
    __builtin_memcpy(xa, &a, 16);
    __builtin_memcpy(xb, &b, 16);
#pragma unroll
    for (int e = 0; e < E; e++) xa[e] = apply<T, OP>(xa[e], xb[e]);
    uint4 r;
    __builtin_memcpy(&r, xa, 16);
    return r;
}

// ---------------------------------------------------------------------------------
// segment kernel
// ---------------------------------------------------------------------------------
constexpr int kBlock = 256;
// 4 x 16 B per lane and operand (16 KiB per operand per workgroup): 6.49-6.50 TB/s on
// rotating buffers with nt stores against 6.14-6.20 for 2 and 6.05-6.09 for 8
// (tools/hbm_sweep.hip, profiles/r02/hbm_sweep_focused.txt)
constexpr int kUnroll = 4;
static_assert(kBlock * kUnroll == kTileVecs, "tile size");

// Streaming operands are read once and results are not re-read by this kernel:
// non-temporal loads AND stores (global_load/store_dwordx4 ... nt).  Timed on rotating
// buffers (tools/hbm_sweep.hip: every launch on one of 4 pairs, 2 GiB, so the 256 MiB
// Infinity Cache holds nothing the next launch reads) the C2 reduce runs at 6.2 TB/s
// with nt stores against 5.6 TB/s with plain ones.  (Round 1's sweep looped over ONE
// pair: there plain stores left the result in the Infinity Cache for the next launch to
// read, which made them look faster -- an artefact of the benchmark, profiles/r02.)
// `nts` is uniform over the launch (FTAR_NT_STORE, default on).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const uint4 *p)
{
    v4u v = __builtin_nontemporal_load((const v4u *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint4 *p, uint4 v, unsigned nts)
{
    if (nts) {
        v4u w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (v4u *)p);
    } else {
        *p = v;
    }
}

// KSignal (ftar_kernels.h): optional acquire before the first load, release + completion
// flag after the last store.  The branch is uniform over the launch.
__device__ __forceinline__ void signal_acquire(const KSignal &G)
{
    if ((G.cnt || G.gate) && G.acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system scope: drop cached remote lines
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// Staging phase of a gated launch (KSignal stage_*): this rank's input copied into its
// exported buffer, element by element (any alignment; a small launch), then released and
// signalled to the host -- all before the gate, which the host opens only after it saw the
// signal and the peers' barrier.  The grid is small (<= FTAR_FLAG_MAX_BLOCKS workgroups), so
// every workgroup is resident while the others wait at the gate.
template <typename E>
__device__ __forceinline__ void stage_copy(const KSignal &G)
{
    const E *s = (const E *)G.stage_src;
    E *d = (E *)G.stage_dst;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < G.stage_n; i += stride) d[i] = s[i];
}

// 16-byte vectors when both ends are 16-byte aligned (the workspace and a hipMalloc'd input
// are), the elements past the last whole vector one by one
__device__ __forceinline__ bool stage_copy_vec(const KSignal &G)
{
    if ((((uintptr_t)G.stage_src | (uintptr_t)G.stage_dst) & 15) != 0) return false;
    const size_t nv = G.stage_n * G.stage_es / 16;
    const uint4 *s = (const uint4 *)G.stage_src;
    uint4 *d = (uint4 *)G.stage_dst;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) d[i] = s[i];
    const size_t done = nv * 16 / G.stage_es; // elements copied as vectors
    if (blockIdx.x == 0)
        for (size_t i = done + threadIdx.x; i < G.stage_n; i += blockDim.x) {
            if (G.stage_es == 8) ((unsigned long long *)G.stage_dst)[i] = ((const unsigned long long *)G.stage_src)[i];
            else ((unsigned *)G.stage_dst)[i] = ((const unsigned *)G.stage_src)[i];
        }
    return true;
}

__device__ __forceinline__ void signal_stage(const KSignal &G)
{
    if (!G.stage_dst) return;
    if (stage_copy_vec(G)) {
    } else if (G.stage_es == 8) stage_copy<unsigned long long>(G);
    else stage_copy<unsigned>(G);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: the staged input to HBM for the peers
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(G.stage_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(G.stage_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(G.flag, G.stage_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The gate of a launch queued ahead of its barrier (KSignal): 1 = run, 0 = skip.  One
// lane polls the host word with system-scope loads (uncached, over PCIe), sleeping
// between polls; the workgroup learns the verdict through LDS.  Uniform over the launch.
// Gates take turns over kGateSlots words (ftar_kernels.h): a workgroup that starts late
// still finds its own verdict after the host has opened the next gate.
// Thread 0: wait until `word` (scope S) reaches the gate's value; skip (and report) past
// `ticks` of the wall clock, or when the word already holds a later gate.
template <int S>
__device__ __forceinline__ unsigned gate_wait(const KSignal &G, const unsigned *word, unsigned long long ticks)
{
    const unsigned long long t0 = wall_clock64();
    unsigned v;
    for (;;) {
        v = __hip_atomic_load(word, __ATOMIC_RELAXED, S);
        if ((int)((v & ~1u) - (G.gate_val & ~1u)) >= 0) break;
        if (wall_clock64() - t0 > ticks) { // the host never opened it: skip, report
            __hip_atomic_store(G.err, G.gate_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v = G.gate_val | 1u;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if ((v & ~1u) != G.gate_val) { // the slot already holds a later gate: never run blind
        __hip_atomic_store(G.err, G.gate_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        v |= 1u;
    }
    return v;
}

__device__ __forceinline__ bool signal_gate(const KSignal &G)
{
    if (G.vword) { // behind a peer wait: its verdict is in device memory already (stream order)
        __shared__ unsigned vgo;
        if (threadIdx.x == 0) vgo = __hip_atomic_load(G.vword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G.vval;
        __syncthreads();
        if (!vgo) return false;
    }
    if (!G.gate) return true;
    __shared__ unsigned go;
    if (threadIdx.x == 0) {
        unsigned v;
        if (!G.gate_dev) {
            v = gate_wait<__HIP_MEMORY_SCOPE_SYSTEM>(G, G.gate, G.gate_ticks);
        } else {
            // relayed: the first workgroup of this gate polls the host word (over PCIe) and
            // relays the verdict through device memory; the others poll that (agent scope)
            const unsigned old = __hip_atomic_fetch_max(G.gate_poll, G.gate_val, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if ((int)(old - G.gate_val) < 0) {
                v = gate_wait<__HIP_MEMORY_SCOPE_SYSTEM>(G, G.gate, G.gate_ticks);
                __hip_atomic_store(G.gate_dev, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                v = gate_wait<__HIP_MEMORY_SCOPE_AGENT>(G, G.gate_dev, 2 * G.gate_ticks);
            }
        }
        go = (v & 1u) ? 0u : 1u;
    }
    __syncthreads();
    return go != 0;
}

__device__ __forceinline__ void signal_done(const KSignal &G)
{
    if (!G.cnt) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this wave's stores have completed
    __syncthreads();                                  // ... and every other wave's
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: this XCD's dirty lines to HBM
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the write-back completed (never elided)
        const unsigned old = __hip_atomic_fetch_add(G.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) { // every workgroup has released: the launch is done
            __hip_atomic_store(G.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(G.flag, G.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename T, int OP>
__device__ __forceinline__ void vec_body(const KSeg &S, size_t b, size_t nblk, unsigned nts)
{
    // Block-contiguous tiles of kBlock * kUnroll vectors (16 KiB per operand per block):
    // each lane issues kUnroll independent 16-byte non-temporal loads per operand, wave
    // instructions stay 1 KiB coalesced, and the grid is sized so that one tile per block
    // covers the segment (the loop only runs when the host capped the grid).
    constexpr size_t E = 16 / sizeof(T);
    constexpr size_t kTile = (size_t)kBlock * kUnroll;
    const uint4 *__restrict__ X = (const uint4 *)S.x;
    const uint4 *__restrict__ Y = (const uint4 *)S.y;
    uint4 *__restrict__ O = (uint4 *)S.out;
    uint4 *__restrict__ O2 = (uint4 *)S.out2; // wave-uniform: both stores or one
    const size_t nv = S.n / E;
    for (size_t base = b * kTile; base < nv; base += nblk * kTile) {
        const size_t i = base + threadIdx.x;
        if (base + kTile <= nv) {
            uint4 a[kUnroll], c[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) a[u] = ldnt(X + i + u * kBlock);
            if (S.kind != kCopy) {
#pragma unroll
                for (int u = 0; u < kUnroll; u++) c[u] = ldnt(Y + i + u * kBlock);
#pragma unroll
                for (int u = 0; u < kUnroll; u++) a[u] = apply16<T, OP>(a[u], c[u]);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; u++) st16(O + i + u * kBlock, a[u], nts);
            if (O2) {
#pragma unroll
                for (int u = 0; u < kUnroll; u++) st16(O2 + i + u * kBlock, a[u], nts);
            }
        } else {
            for (size_t j = i; j < nv; j += kBlock) {
                const uint4 xv = ldnt(X + j);
                const uint4 v = (S.kind == kCopy) ? xv : apply16<T, OP>(xv, ldnt(Y + j));
                st16(O + j, v, nts);
                if (O2) st16(O2 + j, v, nts);
            }
        }
    }
}

template <typename T, int OP>
__device__ __forceinline__ void scalar_body(const KSeg &S, size_t b, size_t nblk)
{
    const T *X = (const T *)S.x;
    const T *Y = (const T *)S.y;
    T *O = (T *)S.out;
    T *O2 = (T *)S.out2;
    const size_t stride = nblk * kBlock;
    for (size_t i = b * kBlock + threadIdx.x; i < S.n; i += stride) {
        const T xv = X[i];
        const T v = (S.kind == kCopy) ? xv : apply<T, OP>(xv, Y[i]);
        O[i] = v;
        if (O2) O2[i] = v;
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void segment_kernel(KSegList L)
{
    // blockIdx is wave-uniform; readfirstlane keeps the lookup in SGPRs.
    const unsigned b = (unsigned)__builtin_amdgcn_readfirstlane((int)blockIdx.x);
    const BlockWork w = map_block(L, b);
    const KSeg &S = L.s[__builtin_amdgcn_readfirstlane(w.seg)];
    signal_stage(L.sig);
    if (signal_gate(L.sig)) {
        signal_acquire(L.sig);
        if (S.vec) vec_body<T, OP>(S, w.first, w.stride, L.nt_store);
        else scalar_body<T, OP>(S, w.first, w.stride);
    }
    signal_done(L.sig);
}

// LDS-DMA staged local reduce (variant 1): the `in` operand is moved HBM -> LDS by
// global_load_lds_dwordx4 (no VGPR destination; 1 KiB per wave instruction, landing at
// the wave-uniform LDS base + 16 B x lane), the `inout` operand comes to VGPRs with
// plain dwordx4 loads issued meanwhile.  Each wave reads back only what it staged, so
// the only ordering needed is the wave's own vmcnt(0) -- no workgroup barrier.
template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void reduce_lds_kernel(uint4 *__restrict__ inout,
                                                            const uint4 *__restrict__ in, size_t nv, unsigned nts)
{
    __shared__ uint4 stage[kUnroll * kBlock]; // 16 KiB per workgroup (kUnroll = 4)
    const int wave = threadIdx.x >> 6;
    const size_t tile = (size_t)kUnroll * kBlock;
    for (size_t base = (size_t)blockIdx.x * tile; base < nv; base += (size_t)gridDim.x * tile) {
        uint4 a[kUnroll];
        if (base + tile <= nv) {
#pragma unroll
            for (int u = 0; u < kUnroll; u++) {
                const uint4 *g = in + base + (size_t)u * kBlock + threadIdx.x;
                uint4 *l = &stage[u * kBlock + wave * 64];
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                                 (__attribute__((address_space(3))) void *)l, 16, 0, 2 /* nt */);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; u++) a[u] = ldnt(inout + base + (size_t)u * kBlock + threadIdx.x);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < kUnroll; u++)
                st16(inout + base + (size_t)u * kBlock + threadIdx.x, apply16<T, OP>(a[u], stage[u * kBlock + threadIdx.x]),
                     nts);
        } else {
            for (size_t i = base + threadIdx.x; i < nv; i += kBlock) st16(inout + i, apply16<T, OP>(inout[i], in[i]), nts);
        }
    }
}

// Tree reduce over p sources (one-hop reduce-scatter on the xGMI mesh): every lane loads
// one 16-byte vector from each of the p sources -- p - 1 of them peers, so all links
// stream at once -- and combines them in the schedule's tree.  Workgroups past the
// vector body take the scalar head/tail (or everything, if the pointers are not
// co-aligned), grid-stride.
// U (1, 2, 4): 16-byte vectors per lane and source, every load of the workgroup's U x P
// vectors issued before the first combine -- more bytes in flight per lane when the
// sources are remote (xGMI load latency) rather than local HBM (FTAR_OPT_TREE_UNROLL; the
// node's transport selection times the forms).  Same tree per element: same bits.
template <typename T, int OP, int P>
__device__ __forceinline__ void tree_store(const TreeArgs &A, size_t i, uint4 (&v)[P])
{
#pragma unroll
    for (int w = 1; w < P; w <<= 1)
#pragma unroll
        for (int j = 0; j < P; j += 2 * w) v[j] = apply16<T, OP>(v[j], v[j + w]);
    st16((uint4 *)((T *)A.out + A.head) + i, v[0], A.nt_store);
    for (int o = 0; o < A.nmore; o++) st16((uint4 *)((T *)A.more[o] + A.head) + i, v[0], A.nt_store);
}

template <typename T, int OP, int P, int U>
__device__ __forceinline__ void tree_body(const TreeArgs &A, unsigned b, unsigned nblocks)
{
    if (b < A.nvb) {
        // chunk b, then b + nvb, ... (once, unless the planner capped the vector workgroups:
        // cap_tree_batch, a gated one-shot launch that must stay within the signal limit)
        for (size_t c = b; c * kBlock * U < A.nv; c += A.nvb) {
            const size_t i0 = c * kBlock * U + threadIdx.x;
            if (i0 + (size_t)(U - 1) * kBlock < A.nv) {
                uint4 v[U][P];
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int j = 0; j < P; j++)
                        v[u][j] = ldnt((const uint4 *)((const T *)A.src[j] + A.head) + i0 + (size_t)u * kBlock);
#pragma unroll
                for (int u = 0; u < U; u++) tree_store<T, OP, P>(A, i0 + (size_t)u * kBlock, v[u]);
            } else {
                for (int u = 0; u < U; u++) {
                    const size_t i = i0 + (size_t)u * kBlock;
                    if (i >= A.nv) break;
                    uint4 v[P];
#pragma unroll
                    for (int j = 0; j < P; j++) v[j] = ldnt((const uint4 *)((const T *)A.src[j] + A.head) + i);
                    tree_store<T, OP, P>(A, i, v);
                }
            }
        }
        return;
    }
    constexpr size_t E = 16 / sizeof(T);
    const size_t tail0 = A.head + A.nv * E; // scalar elements: [0, head) and [tail0, n)
    const size_t nscalar = A.head + (A.n - tail0);
    const size_t stride = (size_t)(nblocks - A.nvb) * kBlock;
    for (size_t k = (size_t)(b - A.nvb) * kBlock + threadIdx.x; k < nscalar; k += stride) {
        const size_t e = k < A.head ? k : tail0 + (k - A.head);
        T v[P];
#pragma unroll
        for (int j = 0; j < P; j++) v[j] = ((const T *)A.src[j])[e];
#pragma unroll
        for (int w = 1; w < P; w <<= 1)
#pragma unroll
            for (int j = 0; j < P; j += 2 * w) v[j] = apply<T, OP>(v[j], v[j + w]);
        ((T *)A.out)[e] = v[0];
        for (int o = 0; o < A.nmore; o++) ((T *)A.more[o])[e] = v[0];
    }
}

template <typename T, int OP, int P, int U>
__global__ __launch_bounds__(kBlock) void tree_kernel(TreeArgs A)
{
    tree_body<T, OP, P, U>(A, (unsigned)__builtin_amdgcn_readfirstlane((int)blockIdx.x), gridDim.x);
}

// Several trees in one launch (the one-shot mesh Allreduce: every block of the vector,
// each in its owner's tree): tree k takes workgroups [first[k], first[k + 1]).
template <typename T, int OP, int P>
__global__ __launch_bounds__(kBlock) void tree_batch_kernel(TreeBatch B)
{
    const unsigned b = (unsigned)__builtin_amdgcn_readfirstlane((int)blockIdx.x);
    int k = 0;
    while (k + 1 < B.nt && b >= B.first[k + 1]) k++;
    signal_stage(B.sig);
    if (signal_gate(B.sig)) {
        signal_acquire(B.sig);
        tree_body<T, OP, P, 1>(B.t[k], b - B.first[k], B.first[k + 1] - B.first[k]);
    }
    signal_done(B.sig);
}

// ---------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------
unsigned plan_tree(TreeArgs *A, int p, size_t esize, unsigned max_blocks)
{
    uintptr_t mis = (uintptr_t)A->out & 15;
    bool co = (16 % esize == 0) && (mis % esize == 0);
    for (int j = 0; j < p; j++) co = co && (((uintptr_t)A->src[j] & 15) == mis);
    for (int o = 0; o < A->nmore; o++) co = co && (((uintptr_t)A->more[o] & 15) == mis);
    A->head = A->nv = 0;
    if (co) {
        size_t head = mis ? (16 - mis) / esize : 0;
        if (head > A->n) head = A->n;
        A->head = head;
        A->nv = (A->n - head) * esize / 16;
    }
    size_t nscalar = A->n - A->nv * (16 / esize);
    const unsigned u = (A->unroll == 2 || A->unroll == 4) && (p == 4 || p == 8) ? A->unroll : 1;
    A->unroll = u;
    size_t vb = (A->nv + (size_t)kBlock * u - 1) / ((size_t)kBlock * u);
    if (vb > max_blocks) return 0; // the caller splits larger blocks
    size_t sb = (nscalar + kBlock - 1) / kBlock;
    if (sb > 256) sb = 256;
    A->nvb = (unsigned)vb;
    return (unsigned)(vb + sb);
}

template <typename T, int OP, int P>
static void launch_tree_u(const TreeArgs &A, unsigned grid, hipStream_t s)
{
    if constexpr (P == 4 || P == 8) {
        if (A.unroll == 4) {
            hipLaunchKernelGGL((tree_kernel<T, OP, P, 4>), dim3(grid), dim3(kBlock), 0, s, A);
            return;
        }
        if (A.unroll == 2) {
            hipLaunchKernelGGL((tree_kernel<T, OP, P, 2>), dim3(grid), dim3(kBlock), 0, s, A);
            return;
        }
    }
    hipLaunchKernelGGL((tree_kernel<T, OP, P, 1>), dim3(grid), dim3(kBlock), 0, s, A);
}

template <typename T, int OP>
static hipError_t launch_tree_op(int p, const TreeArgs &A, unsigned grid, hipStream_t s)
{
    switch (p) {
    case 2: launch_tree_u<T, OP, 2>(A, grid, s); break;
    case 4: launch_tree_u<T, OP, 4>(A, grid, s); break;
    case 8: launch_tree_u<T, OP, 8>(A, grid, s); break;
    case 16: launch_tree_u<T, OP, 16>(A, grid, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_tree_t(int op, int p, const TreeArgs &A, unsigned grid, hipStream_t s)
{
    return with_op<T>(op, [&](auto o) { return launch_tree_op<T, decltype(o)::value>(p, A, grid, s); });
}

hipError_t launch_tree(int dtype, int op, int p, const TreeArgs &A, unsigned grid, hipStream_t s)
{
    switch (dtype) {
    case kInt32: return launch_tree_t<int32_t>(op, p, A, grid, s);
    case kFloat32: return launch_tree_t<float>(op, p, A, grid, s);
    case kInt64: return launch_tree_t<int64_t>(op, p, A, grid, s);
    case kFloat64: return launch_tree_t<double>(op, p, A, grid, s);
    default: return hipErrorInvalidValue;
    }
}
unsigned plan_tree_batch(TreeBatch *B, int p, size_t esize, unsigned max_blocks)
{
    unsigned total = 0;
    for (int k = 0; k < B->nt; k++) {
        B->first[k] = total;
        B->t[k].unroll = 1; // tree_batch_kernel is instantiated for one vector per lane and source
        unsigned g = plan_tree(&B->t[k], p, esize, max_blocks);
        if (g == 0) return 0;
        total += g;
    }
    B->first[B->nt] = total;
    return total;
}

unsigned cap_tree_batch(TreeBatch *B, unsigned max_total)
{
    unsigned sb = 0, vb = 0, trees_v = 0;
    for (int k = 0; k < B->nt; k++) {
        vb += B->t[k].nvb;
        sb += B->first[k + 1] - B->first[k] - B->t[k].nvb;
        trees_v += B->t[k].nvb > 0;
    }
    if (vb + sb <= max_total) return vb + sb;
    if (sb + trees_v > max_total) return 0;
    const unsigned avail = max_total - sb;
    unsigned nvb[kMaxBatch], total = 0;
    for (int k = 0; k < B->nt; k++) {
        nvb[k] = B->t[k].nvb ? (unsigned)((unsigned long long)B->t[k].nvb * avail / vb) : 0;
        if (B->t[k].nvb && nvb[k] < 1) nvb[k] = 1;
        total += nvb[k] + (B->first[k + 1] - B->first[k] - B->t[k].nvb);
    }
    if (total > max_total) return 0; // unchanged
    total = 0;
    for (int k = 0; k < B->nt; k++) {
        const unsigned s = B->first[k + 1] - B->first[k] - B->t[k].nvb;
        B->first[k] = total;
        B->t[k].nvb = nvb[k];
        total += nvb[k] + s;
    }
    B->first[B->nt] = total;
    return total;
}

template <typename T, int OP>
static hipError_t launch_batch_op(int p, const TreeBatch &B, unsigned grid, hipStream_t s)
{
    switch (p) {
    case 2: hipLaunchKernelGGL((tree_batch_kernel<T, OP, 2>), dim3(grid), dim3(kBlock), 0, s, B); break;
    case 4: hipLaunchKernelGGL((tree_batch_kernel<T, OP, 4>), dim3(grid), dim3(kBlock), 0, s, B); break;
    case 8: hipLaunchKernelGGL((tree_batch_kernel<T, OP, 8>), dim3(grid), dim3(kBlock), 0, s, B); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_batch_t(int op, int p, const TreeBatch &B, unsigned grid, hipStream_t s)
{
    return with_op<T>(op, [&](auto o) { return launch_batch_op<T, decltype(o)::value>(p, B, grid, s); });
}

hipError_t launch_tree_batch(int dtype, int op, int p, const TreeBatch &B, unsigned grid, hipStream_t s)
{
    switch (dtype) {
    case kInt32: return launch_batch_t<int32_t>(op, p, B, grid, s);
    case kFloat32: return launch_batch_t<float>(op, p, B, grid, s);
    case kInt64: return launch_batch_t<int64_t>(op, p, B, grid, s);
    case kFloat64: return launch_batch_t<double>(op, p, B, grid, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename T>
static hipError_t launch_t(int op, const KSegList &L, unsigned grid, hipStream_t s)
{
    return with_op<T>(op, [&](auto o) {
        hipLaunchKernelGGL((segment_kernel<T, decltype(o)::value>), dim3(grid), dim3(kBlock), 0, s, L);
        return hipGetLastError();
    });
}

// PeerWait (ftar_kernels.h): one wavefront, lane i < npeers polls peer i's flag.
__global__ __launch_bounds__(64) void peer_wait_kernel(PeerWait W)
{
    const int lane = threadIdx.x;
    if (lane == 0) {
        __hip_atomic_store(W.own, W.token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: the flag out to host memory for the peers
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long *mine = lane < W.npeers ? W.peer[lane] : nullptr;
    const unsigned long long t0 = wall_clock64();
    bool go = false;
    for (;;) {
        const bool ready = !mine || __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= W.token;
        if (__all(ready)) {
            go = true;
            break;
        }
        if (__hip_atomic_load(W.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == W.vval) break;
        if (wall_clock64() - t0 > W.ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
        const unsigned v = go ? W.vval : (W.vval | 1u);
        __hip_atomic_store(W.verdict_dev, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(W.verdict_host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_peer_wait(const PeerWait &W, hipStream_t s)
{
    if (W.npeers < 1 || W.npeers > kMaxPeers || !W.own || !W.abort_word || !W.verdict_dev || !W.verdict_host)
        return hipErrorInvalidValue;
    for (int i = 0; i < W.npeers; i++)
        if (!W.peer[i]) return hipErrorInvalidValue;
    hipLaunchKernelGGL(peer_wait_kernel, dim3(1), dim3(64), 0, s, W);
    return hipGetLastError();
}

hipError_t launch_segments(int dtype, int op, const KSegList &L, unsigned grid, hipStream_t s)
{
    switch (dtype) {
    case kInt32: return launch_t<int32_t>(op, L, grid, s);
    case kFloat32: return launch_t<float>(op, L, grid, s);
    case kInt64: return launch_t<int64_t>(op, L, grid, s);
    case kFloat64: return launch_t<double>(op, L, grid, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename T>
static hipError_t launch_lds_t(int op, uint4 *inout, const uint4 *in, size_t nv, unsigned grid, hipStream_t s,
                               unsigned nts)
{
    return with_op<T>(op, [&](auto o) {
        hipLaunchKernelGGL((reduce_lds_kernel<T, decltype(o)::value>), dim3(grid), dim3(kBlock), 0, s, inout, in, nv,
                           nts);
        return hipGetLastError();
    });
}

hipError_t launch_reduce_lds(int dtype, int op, void *inout, const void *in, size_t nvec, unsigned grid,
                             hipStream_t s, unsigned nts)
{
    uint4 *io = (uint4 *)inout;
    const uint4 *i = (const uint4 *)in;
    switch (dtype) {
    case kInt32: return launch_lds_t<int32_t>(op, io, i, nvec, grid, s, nts);
    case kFloat32: return launch_lds_t<float>(op, io, i, nvec, grid, s, nts);
    case kInt64: return launch_lds_t<int64_t>(op, io, i, nvec, grid, s, nts);
    case kFloat64: return launch_lds_t<double>(op, io, i, nvec, grid, s, nts);
    default: return hipErrorInvalidValue;
    }
}

// Split user segments into co-aligned vector bodies + scalar heads/tails and assign
// blocks.  Returns the grid size (0 if there is nothing to do).
unsigned plan_segments(const SegIn *in, int nin, size_t esize, unsigned max_blocks, KSegList *L)
{
    L->nseg = 0;
    L->nt_store = 0;
    L->sig = KSignal{nullptr, nullptr, 0, 0};
    size_t vec_bytes_total = 0;
    struct Piece { KSeg k; size_t bytes; } pieces[kMaxKSegs];
    int np = 0;
    for (int s = 0; s < nin; s++) {
        const SegIn &g = in[s];
        if (g.n == 0) continue;
        uintptr_t ao = (uintptr_t)g.out, ax = (uintptr_t)g.x, ay = (uintptr_t)(g.kind == kCopy ? g.x : g.y);
        uintptr_t ao2 = g.out2 ? (uintptr_t)g.out2 : ao;
        bool co = ((ao & 15) == (ax & 15)) && ((ao & 15) == (ay & 15)) && ((ao & 15) == (ao2 & 15)) &&
                  (16 % esize == 0) && ((ao & 15) % esize == 0);
        size_t head = 0, body = 0;
        if (co) {
            size_t mis = ao & 15;
            head = mis ? (16 - mis) / esize : 0;
            if (head > g.n) head = g.n;
            size_t rest = g.n - head;
            size_t epv = 16 / esize;
            body = (rest / epv) * epv;
        }
        size_t tail_off = head + body;
        auto add = [&](size_t off, size_t n, unsigned vec) {
            if (n == 0) return;
            KSeg k;
            k.out = (char *)g.out + off * esize;
            k.out2 = g.out2 ? (void *)((char *)g.out2 + off * esize) : nullptr;
            k.x = (const char *)g.x + off * esize;
            k.y = g.kind == kCopy ? k.x : (const void *)((const char *)g.y + off * esize);
            k.n = n;
            k.kind = (unsigned)g.kind;
            k.vec = vec;
            k.blk_begin = k.blk_end = 0;
            pieces[np].k = k;
            pieces[np].bytes = n * esize;
            if (vec) vec_bytes_total += n * esize;
            np++;
        };
        add(0, head, 0);
        add(head, body, 1);
        add(tail_off, g.n - tail_off, 0);
    }
    if (np == 0) return 0;
    const size_t tile_bytes = (size_t)kBlock * 16 * kUnroll;
    size_t total_tiles = 0;
    for (int i = 0; i < np; i++)
        if (pieces[i].k.vec) total_tiles += (pieces[i].bytes + tile_bytes - 1) / tile_bytes;
    L->nil = 0;
    L->il_blocks = 0;
    if (total_tiles + 64 * (size_t)np <= max_blocks) {
        // uncapped grid: one block per tile.  Vector pieces of at least one chunk share
        // an interleaved prefix of `rounds` chunks each (the shortest one's length).
        size_t rounds = SIZE_MAX;
        unsigned char il[kMaxIleave];
        int nil = 0;
        for (int i = 0; i < np && nil < kMaxIleave; i++) {
            if (!pieces[i].k.vec) continue;
            size_t t = (pieces[i].bytes + tile_bytes - 1) / tile_bytes;
            if (t < (size_t)kChunkTiles) continue;
            il[nil++] = (unsigned char)i;
            if (t / kChunkTiles < rounds) rounds = t / kChunkTiles;
        }
        if (nil >= 2) {
            L->nil = nil;
            L->il_blocks = (unsigned)(rounds * kChunkTiles * nil);
            memcpy(L->il, il, sizeof(il));
        } else {
            rounds = 0;
        }
        unsigned next = L->il_blocks;
        for (int i = 0; i < np; i++) {
            KSeg &k = pieces[i].k;
            bool in_il = false;
            for (int t = 0; t < L->nil; t++) in_il |= (L->il[t] == i);
            size_t tiles = k.vec ? (pieces[i].bytes + tile_bytes - 1) / tile_bytes : 0;
            size_t base = in_il ? rounds * kChunkTiles : 0;
            size_t want = k.vec ? tiles - base : (k.n + kBlock - 1) / kBlock;
            if (!k.vec && want > 64) want = 64;
            k.ntiles = (unsigned)tiles;
            k.tile_base = (unsigned)base;
            k.blk_begin = next;
            k.blk_end = next + (unsigned)want;
            next = k.blk_end;
            L->s[L->nseg++] = k;
        }
        return next;
    }
    // capped grid (more than max_blocks tiles): blocks split between the pieces in
    // proportion to their bytes, pieces loop with a block stride; scalar pieces (heads/
    // tails < 16 B, or non-co-aligned slow paths) get up to 64 blocks.
    unsigned next = 0;
    for (int i = 0; i < np; i++) {
        KSeg &k = pieces[i].k;
        size_t want;
        if (k.vec) {
            size_t need = (pieces[i].bytes + tile_bytes - 1) / tile_bytes;
            size_t share = vec_bytes_total ? (size_t)((double)max_blocks * (double)pieces[i].bytes /
                                                     (double)vec_bytes_total) + 1
                                           : 1;
            want = need < share ? need : share;
            k.ntiles = (unsigned)need;
        } else {
            size_t need = (k.n + kBlock - 1) / kBlock;
            want = need < 64 ? need : 64;
            k.ntiles = 0;
        }
        if (want < 1) want = 1;
        k.tile_base = 0;
        k.blk_begin = next;
        k.blk_end = next + (unsigned)want;
        next = k.blk_end;
        L->s[L->nseg++] = k;
    }
    return next;
}

} // namespace ftar
