// ftar_kernels.h -- internal interface between the HIP runtime glue and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace ftar {

enum { kInt32 = 0, kFloat32 = 1, kInt64 = 2, kFloat64 = 3 };
enum { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kLand = 4, kBand = 5, kLor = 6, kBor = 7, kLxor = 8, kBxor = 9 };
constexpr int kNumOps = 10; // logical / bitwise ops (>= kLand) exist for the integer types only
enum { kCopy = 0, kReduce = 1 };

constexpr int kMaxKSegs = 48; // 16 user segments x (head, body, tail); 2.3 KB of kernarg
constexpr int kTileVecs = 1024; // 16-byte vectors per workgroup tile (256 threads x 4)
constexpr int kChunkTiles = 8; // tiles per chunk of the interleaved block mapping (128 KiB)
constexpr int kMaxIleave = 16; // vector pieces that can share the interleaved prefix

// Completion signal of a short launch (the small-message path): instead of a
// marker packet the host spins on, the kernel itself tells the host it is done.  Every
// workgroup, once its stores have completed, releases them at system scope (write-back of
// its XCD's L2: the data is in HBM for peer GPUs and the host) and adds one to `cnt`; the
// workgroup whose add completes the grid resets `cnt` and stores `tag` into `flag`, a word of
// pinned host memory the host polls.  `acquire`: every workgroup first invalidates its
// cached copies of remote memory (system-scope acquire) -- the host sets it when the last
// drain was such a signal, i.e. no marker packet has invalidated the caches since the
// barrier after which this launch reads the peers' new data.
//
// `gate` (optional): the launch was queued before the host barrier that makes its
// operands ready.  Thread 0 of every workgroup polls the pinned host word (system scope)
// until it reaches gate_val (= 2 x sequence, bit 0 set = skip), the workgroup then runs or
// returns without touching memory; either way it signals.  A gate still closed after
// gate_ticks of the wall clock (tens of seconds: the host never got past its barrier) is
// taken as skip and reported through `err`, which the host checks after the drain.
constexpr unsigned kGateSlots = 8; // gate words, used in turn (sig_flag[16 + seq % 8])
struct KSignal {
    unsigned *cnt;  // device counter, agent-scope atomics; nullptr = no signal
    unsigned *flag; // pinned host word
    unsigned tag;
    unsigned acquire;
    const unsigned *gate; // pinned host word (slot gate_val / 2 % kGateSlots); nullptr = not gated
    unsigned gate_val;
    unsigned *err;        // pinned host word of this gate's slot: set to gate_val on a gate timeout
    unsigned long long gate_ticks;
    // Relayed gate (every gated launch of FTAR_GATE_RELAY_MIN = 2 workgroups or more: the short
    // signalling ones and the mid-size ones queued behind a fenced marker): only the first
    // workgroup to start -- elected by an atomic max of gate_val into *gate_poll -- polls the
    // host word over PCIe; it relays the verdict through the device word *gate_dev, which the
    // other workgroups poll.  nullptr = the workgroup polls the host word itself.
    unsigned *gate_poll;
    unsigned *gate_dev;
    // Optional staging phase BEFORE the gate (a gated launch that also stages this rank's
    // input for its peers, saving the separate staging launch): every workgroup copies its
    // share of stage_n elements of stage_es bytes from stage_src to stage_dst, releases its
    // stores at system scope and counts itself in stage_cnt; the last one stores stage_tag
    // into `flag` -- the host's signal that the input is staged, before it opens the gate.
    const void *stage_src;
    void *stage_dst;
    size_t stage_n;
    unsigned stage_es;
    unsigned stage_tag;
    unsigned *stage_cnt;  // device counter (agent scope)
    // Behind a peer wait (PeerWait, queued just before on the same stream): every workgroup
    // runs only if the wait kernel wrote `vval` into the device word *vword (go); any other
    // value (vval | 1: given up) and it returns untouched.  nullptr = no wait in front.
    const unsigned *vword;
    unsigned vval;
};

// The wait of the mesh allgather for the peers' reduce-scatter (fdev_peer_wait): ONE
// wavefront.  Lane 0 first publishes this rank's flag (`token` into *own, system scope: the
// flags are lines of one host page every rank's GPU maps, read coherently by every GPU of the
// node; the tree's data was released to HBM device-wide by the fenced marker in front of this
// kernel); then lane i polls peer i's flag over PCIe (system-scope loads of host memory)
// until every one holds at least `token`, the host's abort word holds vval (a peer died: give
// up), or `ticks` of the wall clock pass (give up, so the grid always drains).  The verdict
// (vval = go, vval | 1 = given up) goes to *verdict_dev for the launch behind it and to the
// pinned host word *verdict_host for the host after its drain.
constexpr int kMaxPeers = 15;
struct PeerWait {
    unsigned long long *own;
    const unsigned long long *peer[kMaxPeers];
    int npeers;
    unsigned long long token;
    const unsigned *abort_word;
    unsigned *verdict_dev;
    unsigned *verdict_host;
    unsigned vval;
    unsigned long long ticks;
};
hipError_t launch_peer_wait(const PeerWait &W, hipStream_t s);

struct KSeg {
    void *out;
    void *out2;          // optional second destination (same values), nullptr = none
    const void *x;
    const void *y;
    size_t n;
    unsigned kind;
    unsigned vec;
    unsigned blk_begin;  // sequential region: blocks [blk_begin, blk_end) ...
    unsigned blk_end;
    unsigned tile_base;  // ... take tiles tile_base, tile_base + 1, ... of this piece
    unsigned ntiles;     // tiles of the whole piece (the stride of a capped grid)
};

// Blocks [0, il_blocks) are dealt round-robin, one kChunkTiles chunk at a time, over the
// vector pieces il[0..nil): pieces that pull from different peers then stream over
// their xGMI links at the same time instead of one after the other.  The remaining
// blocks map sequentially (blk_begin/blk_end) onto what is left of every piece.
struct KSegList {
    KSeg s[kMaxKSegs];
    int nseg;
    int nil;
    unsigned il_blocks;
    unsigned char il[kMaxIleave];
    unsigned nt_store; // 16-byte stores non-temporal (set by the caller after plan_segments)
    KSignal sig;       // optional completion signal (sig.cnt == nullptr: none)
};

// What one workgroup of segment_kernel processes: piece `seg`, starting at tile (vector
// pieces) or block slot (scalar pieces) `first`, then every `stride`-th one.  Shared by
// the kernel and the host-side coverage test (tests/kernel_plan).
struct BlockWork {
    int seg;
    size_t first;
    size_t stride;
};

__host__ __device__ inline BlockWork map_block(const KSegList &L, unsigned b)
{
    BlockWork w;
    if (b < L.il_blocks) { // interleaved prefix: chunk q of piece il[q % nil]
        const unsigned q = b / kChunkTiles;
        w.seg = L.il[q % (unsigned)L.nil];
        w.first = (size_t)(q / (unsigned)L.nil) * kChunkTiles + b % kChunkTiles;
        w.stride = L.s[w.seg].ntiles;
        return w;
    }
    int si = 0;
    while (si + 1 < L.nseg && b >= L.s[si].blk_end) si++;
    const KSeg &S = L.s[si];
    const size_t j = b - S.blk_begin, nblk = S.blk_end - S.blk_begin;
    w.seg = si;
    w.first = (S.vec ? S.tile_base : 0) + j;
    w.stride = (S.vec && S.tile_base) ? S.ntiles : nblk;
    return w;
}

struct SegIn {
    int kind;
    void *out;
    const void *x;
    const void *y;
    size_t n;
    void *out2;
};

// Tree reduce: out[i] = balanced left-to-right tree of src[0..p-1][i] (p = 2, 4, 8, 16):
// ((s0 op s1) op (s2 op s3)) op ...  With the sources in owner-relative order
// (src[j] = vrank owner ^ j) this is exactly the value recursive halving leaves in the
// owner's final block (every level: the owner's subtree first).
constexpr int kMaxTree = 16;
constexpr int kMaxMore = 7; // extra destinations of one tree (the push mesh's allgather: every peer)
struct TreeArgs {
    const void *src[kMaxTree];
    void *out;
    void *more[kMaxMore]; // further destinations receiving the same values (nmore of them)
    int nmore;
    size_t n;      // elements
    size_t head;   // scalar elements before the 16-byte vector body (co-aligned sources)
    size_t nv;     // 16-byte vectors in the body (0 when the pointers are not co-aligned)
    unsigned nvb;  // workgroups of the vector body; the rest do the scalar elements
    unsigned nt_store; // 16-byte stores non-temporal
    unsigned unroll;   // 16-byte vectors per lane and source (1, 2, 4; > 1 only for tree_kernel at p = 4, 8)
};
constexpr int kMaxUnroll = 4;
// fills the alignment fields of A (src/out/n/unroll set) and returns the grid size
unsigned plan_tree(TreeArgs *A, int p, size_t esize, unsigned max_blocks);
hipError_t launch_tree(int dtype, int op, int p, const TreeArgs &A, unsigned grid, hipStream_t s);
// up to kMaxBatch trees of p <= kMaxBatchP sources in one launch; tree k owns
// workgroups [first[k], first[k + 1])
constexpr int kMaxBatch = 8, kMaxBatchP = 8;
struct TreeBatch {
    TreeArgs t[kMaxBatch];
    unsigned first[kMaxBatch + 1];
    int nt;
    KSignal sig; // optional completion signal
};
unsigned plan_tree_batch(TreeBatch *B, int p, size_t esize, unsigned max_blocks);
// shrinks a planned batch to at most max_total workgroups by giving each vector workgroup
// several chunks (its scalar workgroups stay); the new grid, or 0 if it cannot fit
unsigned cap_tree_batch(TreeBatch *B, unsigned max_total);
hipError_t launch_tree_batch(int dtype, int op, int p, const TreeBatch &B, unsigned grid, hipStream_t s);

unsigned plan_segments(const SegIn *in, int nin, size_t esize, unsigned max_blocks, KSegList *L);
hipError_t launch_segments(int dtype, int op, const KSegList &L, unsigned grid, hipStream_t s);
hipError_t launch_reduce_lds(int dtype, int op, void *inout, const void *in, size_t nvec, unsigned grid,
                             hipStream_t s, unsigned nt_store);

} // namespace ftar
