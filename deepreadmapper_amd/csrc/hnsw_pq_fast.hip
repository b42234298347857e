// deepreadmapper_amd/csrc/hnsw_pq_fast.hip -- lean HNSW-PQ search kernel for the common shape
// (PQ 8 x 8 bits, level-0 degree <= 64, ef <= 128), bit-identical to the exact kernel in
// hnsw_search.hip and to the oracle (faiss IndexHNSW::search -> HNSW::search ->
// search_from_candidates with MinimaxHeap + HeapBlockResultHandler [upstream faiss >= 1.8],
// restated in oracle/drm_oracle.c). Caller: faiss_search (src/hnswpq/search.cpp:39-40).
//
// What makes it lean ("hnsw_pq_fast_kernel"):
//   * every MinimaxHeap slot is one u64 = (ord32(distance) << 32) | (id ^ 2^31): faiss's cmp2 on
//     (distance, id) -- popped slots carry id -1 -- becomes a single unsigned 64-bit compare;
//   * the heap sits in the sibling-pair layout (lane p holds the children of node p, slots 2p+1 and
//     2p+2; the root is lane 63's second half); a full-heap replace finds its sift-down path from two
//     ballots and per-lane ancestor masks, and its sift-up chain by one parallel compare;
//   * pop_min checks the previous hop's prediction of the minimum with two ballots (a 32-bit DPP min
//     only when it missed) and takes the highest tied slot from lane masks;
//   * result set at k == ef: the HeapBlockResultHandler (k = ef) holds, at every step, the same
//     multiset of distances as the MinimaxHeap, and the heap slots carry node ids, so the k results are
//     the heap's entries plus the evicted ones that tied with the root they left (a log of those alone);
//     selected + sorted once per query. k < ef keeps a register result set (k <= 64);
//   * no visited table. faiss's VisitedTable answers "was this link seen before?"; the kernel answers it
//     from the heap instead ("The heap is the visited set"). Every heap slot also
//     carries its node id (IL / IR), popped or not. A link whose distance is at or above the root of the
//     full heap is rejected by MinimaxHeap::push whether it was seen or not (the root only falls), and a
//     seen link below that root has never left the heap; so "seen" == "in the heap" wherever it decides
//     anything, and the same pushes are accepted in the same order as with faiss's table. The hop's only
//     memory access is its level-0 row (ids + codes inline), predicted and fetched one hop ahead.
//     ndis (faiss's count of never-seen links) needs the table: the STATS instantiation keeps a plain
//     bitmap beside the heap for the count only (drm_index_set_exact_stats).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "drm_device.h"
#include "pq_common.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

constexpr uint32_t kPopLo = 0x7FFFFFFFu;            // low word of a popped slot (id -1 ^ 2^31)
constexpr uint64_t kUnused = 0xFFFFFFFF7FFFFFFFull; // key above every distance, popped

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint64_t pack(uint32_t key, int32_t id)
{
    return ((uint64_t)key << 32) | (uint32_t)((uint32_t)id ^ 0x80000000u);
}
__device__ __forceinline__ uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }
__device__ __forceinline__ uint32_t lo32(uint64_t v) { return (uint32_t)v; }
__device__ __forceinline__ int32_t unpack_id(uint64_t v) { return (int32_t)(lo32(v) ^ 0x80000000u); }
__device__ __forceinline__ int32_t readlane32(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
// llvm.amdgcn.writelane (this clang has no builtin for it): old with lane `lane` (wave-uniform, mod 64) replaced by
// the wave-uniform val -- one v_writelane_b32, no compare and no copy of val into a VGPR
extern "C" __device__ int drm_llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ int32_t writelane32(int32_t v, int32_t s, uint32_t l)
{
    return drm_llvm_writelane(s, (int)(l & 63u), v);
}
__device__ __forceinline__ uint64_t writelane64(uint64_t v, uint64_t s, uint32_t l)
{
    const uint32_t h = (uint32_t)drm_llvm_writelane((int)(s >> 32), (int)(l & 63u), (int)(v >> 32));
    const uint32_t o = (uint32_t)drm_llvm_writelane((int)(uint32_t)s, (int)(l & 63u), (int)(uint32_t)v);
    return ((uint64_t)h << 32) | o;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)hi32(v), l);
    const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)lo32(v), l);
    return ((uint64_t)h << 32) | o;
}
__device__ __forceinline__ uint32_t bperm32(uint32_t v, int src)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src)
{
    return ((uint64_t)bperm32(hi32(v), src) << 32) | bperm32(lo32(v), src);
}
__device__ __forceinline__ int32_t bperm32_addr(int32_t v, uint32_t addr) // addr = source lane * 4
{
    return __builtin_amdgcn_ds_bpermute((int)addr, v);
}
__device__ __forceinline__ uint64_t bperm64_addr(uint64_t v, uint32_t addr)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)hi32(v)) << 32) |
           (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)lo32(v));
}
// a wave-uniform lane mask as this lane's predicate, with no per-lane arithmetic (the select uses the mask)
__device__ __forceinline__ bool in_mask(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ int bitlen(uint32_t x) { return 32 - __builtin_clz(x); } // x >= 1
__device__ __forceinline__ uint32_t dpp_rol1_u32(uint32_t v) // lane i <- lane i+1, lane 63 <- lane 0 (wave_rol:1)
{
    // every lane is written (a rotate), so no "old" value: mov_dpp leaves it undefined, and the v_mov that would
    // initialise it goes
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t dpp_shr1_u64(uint64_t old, uint64_t v) // lane i <- lane i-1
{
    const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp((int)hi32(old), (int)hi32(v), 0x138, 0xF, 0xF, false);
    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp((int)lo32(old), (int)lo32(v), 0x138, 0xF, 0xF, false);
    return ((uint64_t)h << 32) | o;
}

// byte M of c times 4 (the LUT entry's byte offset within its sub-quantizer row) in one SDWA shift
template <int M>
__device__ __forceinline__ uint32_t bx4(uint32_t c)
{
    uint32_t r;
    if constexpr (M == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(c));
    else if constexpr (M == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(c));
    else if constexpr (M == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(c));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(c));
    return r;
}

// PQ-ADC distance of one 8-byte code per lane: the 8 LUT reads (sub-quantizer m at byte offset m * 1024) all in
// flight before the first add, then the adds in sub-quantizer order (distance_to_code, 0 ulp vs the oracle)
__device__ __forceinline__ uint32_t adc8(const float *lut, uint2 c)
{
    const char *b = reinterpret_cast<const char *>(lut);
    float lv[8];
    lv[0] = *reinterpret_cast<const float *>(b + bx4<0>(c.x));
    lv[1] = *reinterpret_cast<const float *>(b + bx4<1>(c.x) + 1024);
    lv[2] = *reinterpret_cast<const float *>(b + bx4<2>(c.x) + 2048);
    lv[3] = *reinterpret_cast<const float *>(b + bx4<3>(c.x) + 3072);
    lv[4] = *reinterpret_cast<const float *>(b + bx4<0>(c.y) + 4096);
    lv[5] = *reinterpret_cast<const float *>(b + bx4<1>(c.y) + 5120);
    lv[6] = *reinterpret_cast<const float *>(b + bx4<2>(c.y) + 6144);
    lv[7] = *reinterpret_cast<const float *>(b + bx4<3>(c.y) + 7168);
    __builtin_amdgcn_sched_barrier(0);
    // faiss sums from +0.0; +0.0 + x == x for every LUT entry (a sum of squares from +0.0: never -0.0), so the sum
    // starts at the first entry (one add fewer, the same bits)
    float r = lv[0];
#pragma unroll
    for (int m = 1; m < 8; ++m)
        r = __fadd_rn(r, lv[m]);
    // ord32 of a sum of non-negative LUT entries (squared sub-distances, summed from +0.0): the sign bit is clear,
    // so ord32(r) is r's bit pattern with the sign bit set -- one op instead of ord32's select
    return __float_as_uint(r) | 0x80000000u;
}

// Per-lane constants of node p = lane: A = p and its ancestors, Aup = its ancestors, Lreq = the
// ancestors whose path toward p takes the left child (2a + 1).
struct PathConst {
    // every ancestor of any lane p (< 64) is below lane 32, so A's, Aup's and Lreq's high halves hold at most p
    // itself: the low halves are kept, and Ahi is p's own bit for p >= 32 (0 below)
    uint32_t Alo, Ahi, Auplo, Lreqlo;
    // ds_bpermute byte addresses: this lane's left / right child lane (slots 2p+1, 2p+2 are held by lanes 2p+1, 2p+2
    // mod 64), and its parent in the chain of slot 127's ancestors (lane >> 1)
    uint32_t addrL, addrR, addrHalf, half; // half = lane >> 1
    // heap filling (push_fill): this lane's halves are the 1-based positions xL = 2p+2 and 2p+3 (lane 63's R: the root,
    // position 1), both of bit length bl; their father is slot p, held by lane (p-1)/2 (its L half when p is odd, its
    // R half when p is even) and, for p = 0, by lane 63's R (the root)
    uint32_t xL, bl, addrF;
    // full-heap push: the chain index of this lane's L half on slot 127's ancestor chain (slot 127 = 0, 63 = 1, 31 = 2,
    // 15 = 3, 7 = 4, 3 = 5, 1 = 6: lanes 63, 31, 15, 7, 3, 1, 0; the root, lane 63's R, is 7); 15 for every other lane
    uint32_t cidx;
    __device__ explicit PathConst(int lane)
        : addrL((uint32_t)((2 * lane + 1) & 63) << 2), addrR((uint32_t)((2 * lane + 2) & 63) << 2),
          addrHalf((uint32_t)(lane >> 1) << 2), half((uint32_t)lane >> 1), xL(2u * (uint32_t)lane + 2u),
          bl((uint32_t)bitlen(2u * (uint32_t)lane + 2u)), addrF(lane > 0 ? (uint32_t)((lane - 1) >> 1) << 2 : 63u << 2),
          cidx(((lane + 1) & lane) == 0 ? 6u - (uint32_t)(31 - __builtin_clz((uint32_t)lane + 1u)) : 15u)
    {
        uint64_t A = 1ull << lane, Aup = 0, Lreq = 0;
        for (int c = lane; c > 0;) {
            const int a = (c - 1) >> 1;
            A |= 1ull << a;
            Aup |= 1ull << a;
            if (c & 1)
                Lreq |= 1ull << a;
            c = a;
        }
        Alo = (uint32_t)A;
        Ahi = (uint32_t)(A >> 32);
        Auplo = (uint32_t)Aup;
        Lreqlo = (uint32_t)Lreq;
    }
    // the lanes on the sift-down path: p and all its ancestors have mv set, and every ancestor chose the child toward
    // p (lm: the nodes that take their L child). One per-lane test and one ballot, no scalar mask arithmetic.
    __device__ __forceinline__ uint64_t path(uint64_t mv, uint64_t lm) const
    {
        const uint32_t x = (~(uint32_t)mv & Alo) | (((uint32_t)lm ^ Lreqlo) & Auplo) | (~(uint32_t)(mv >> 32) & Ahi);
        return ballot(x == 0u);
    }
};

// MinimaxHeap arrays (ef <= 128) in the sibling-pair layout. L / R are the faiss keys (a popped slot's id is -1
// there, as in faiss's ids[] array); IL / IR hold each slot's node id, popped or not (-1: never filled), and move
// with their keys through every sift. They are what the kernel's visited test reads. Lane 63's R / IR is the root.
struct Heap {
    uint64_t L, R;
    int32_t IL, IR;

    // value / node id of slot s (wave-uniform s)
    __device__ __forceinline__ uint64_t get(int s) const
    {
        if (s == 0)
            return readlane64(R, 63);
        const int o = (s - 1) >> 1;
        return (s & 1) ? readlane64(L, o) : readlane64(R, o);
    }
    __device__ __forceinline__ int32_t get_id(int s) const
    {
        if (s == 0)
            return readlane32(IR, 63);
        const int o = (s - 1) >> 1;
        return (s & 1) ? readlane32(IL, o) : readlane32(IR, o);
    }
    // node v is in the heap (one compare per half, wave-uniform answer)
    __device__ __forceinline__ bool holds(int32_t v) const { return (ballot(IL == v) | ballot(IR == v)) != 0ull; }
    // the root's key (high word) and node id
    __device__ __forceinline__ uint32_t root_hi() const { return (uint32_t)__builtin_amdgcn_readlane((int)hi32(R), 63); }
    __device__ __forceinline__ int32_t root_id() const { return readlane32(IR, 63); }

    // faiss heap_pop<CMax<float, int>>(k): slot k-1 sifted down from the root (1-based k >= 1).
    __device__ __forceinline__ void pop(int k, int lane)
    {
        const uint64_t val = get(k - 1);
        const int32_t valI = get_id(k - 1);
        const bool has_l = 2 * lane + 1 <= k - 1;
        const bool has_r = 2 * lane + 2 <= k - 1 && lane != 63;
        const bool takeL = !has_r || L > R;                 // (i2 == k + 1) || cmp2(heap[i1], heap[i2])
        const int ch = takeL ? 2 * lane + 1 : 2 * lane + 2; // chosen child slot
        const uint64_t chv = takeL ? L : R;
        const int32_t chI = takeL ? IL : IR;
        const bool moves = has_l && !(val > chv);           // the child moves up unless cmp2(val, child)
        // next hole position, pointer-doubled: n8(0) is the final hole (depth <= 7)
        const int n1 = moves ? ch : lane;
        int n = n1;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int t = (int)bperm32((uint32_t)n, n & 63);
            n = n < 64 ? t : n;
        }
        const int hole = __builtin_amdgcn_readlane(n, 0);
        // lanes strictly above the hole on its root path moved their chosen child up
        const uint32_t hx = (uint32_t)hole + 1u;
        const int sh = bitlen(hx) - bitlen((uint32_t)lane + 1u);
        const bool writer = sh > 0 && (hx >> sh) == (uint32_t)lane + 1u;
        const uint64_t up = bperm64(chv, ch & 63);
        const int32_t upI = (int32_t)bperm32((uint32_t)chI, ch & 63);
        const bool at_hole = ch == hole;
        const uint64_t nv = at_hole ? val : up;
        const int32_t nvI = at_hole ? valI : upI;
        if (writer && takeL) {
            L = nv;
            IL = nvI;
        }
        if (writer && !takeL) {
            R = nv;
            IR = nvI;
        }
        const bool root_moved = hole != 0;
        const uint64_t rootv = root_moved ? readlane64(chv, 0) : val;
        const int32_t rootI = root_moved ? readlane32(chI, 0) : valI;
        if (lane == 63) {
            R = rootv;
            IR = rootI;
        }
    }

    // faiss heap_push<CMax<float, int>>(k, val): val enters at slot k-1 and sifts up (1-based k >= 1).
    __device__ __forceinline__ void push(int k, uint64_t val, int32_t valI, int lane)
    {
        // lane j in [1, 7] looks at the ancestor a_j = k >> j (1-based)
        const int aj = (lane >= 1 && lane < 8) ? (k >> lane) : 0;
        const int t = aj - 1; // its slot
        const int owner = t <= 0 ? 63 : (t - 1) >> 1;
        const bool sideR = t <= 0 || !(t & 1);
        const uint64_t fl = bperm64(L, owner), fr = bperm64(R, owner);
        const int32_t flI = (int32_t)bperm32((uint32_t)IL, owner), frI = (int32_t)bperm32((uint32_t)IR, owner);
        const uint64_t av = sideR ? fr : fl;
        const int32_t avI = sideR ? frI : flI;
        const bool moves = aj >= 1 && val > av; // cmp2(val, father): the father moves down
        const int h = __builtin_popcountll(ballot(moves)); // ancestors 1..h move (heap order: a prefix)
        // chain index m (a_m = k >> m, m = 0..h) gets a_{m+1}'s value, or val at m == h
        const int bk = bitlen((uint32_t)k);
        const uint32_t xl = 2u * (uint32_t)lane + 2u, xr = xl + 1u; // 1-based indices of L, R
        const int ml = bk - bitlen(xl), mr = bk - bitlen(xr);
        const bool onL = ml >= 0 && ml <= h && (uint32_t)(k >> ml) == xl;
        const bool onR = lane != 63 && mr >= 0 && mr <= h && (uint32_t)(k >> mr) == xr;
        const int m = onL ? ml : mr;
        const uint64_t pulled = bperm64(av, (m + 1) & 63);
        const int32_t pulledI = (int32_t)bperm32((uint32_t)avI, (m + 1) & 63);
        const uint64_t nv = (m == h) ? val : pulled;
        const int32_t nvI = (m == h) ? valI : pulledI;
        if (onL) {
            L = nv;
            IL = nvI;
        }
        if (onR) {
            R = nv;
            IR = nvI;
        }
        // the root (lane 63 R, 1-based 1 = a_{bk-1}) changes only if val climbs all the way up
        if (h == bk - 1 && lane == 63) {
            R = val;
            IR = valI;
        }
    }

    // heap_pop(128) then heap_push(128, vnew) on the full ef = 128 heap (MinimaxHeap::push when k == n), with the
    // cross-lane fetches issued together from the pre-pop registers: one ds_bpermute round trip per replace.
    //  * pop: slot 127 (lane 63's L) is sifted down from the root. Lane p on the path writes its chosen child slot
    //    with that child's own chosen child (chv of lane ch_p), or with slot 127's value when p is the path's last
    //    node; the path is the set of lanes whose own and ancestors' chosen children move up (PathConst::path). The
    //    root (lane 63's R) takes node 0's chosen child when node 0 is on the path, else slot 127's value: lane 0
    //    forms it and lane 63 takes it by one DPP wave rotate;
    //  * push: vnew enters slot 127 and climbs the chain of its ancestors (slots 63, 31, 15, 7, 3, 1: the L halves
    //    of lanes 31, 15, 7, 3, 1, 0; then the root). Chain holder c takes its father, slot c, whose post-pop value
    //    is lane c's own chv (or slot 127's value) if lane c >> 1 is on the path and took its L child, else its
    //    pre-pop value; lane 0's father is the root.
    // Straight-line, and every decision is a per-lane test on the vector unit (the scalar unit only counts h and
    // combines two masks): the scalar-issue share of the hop is what bounds the kernel. The
    // caller reads the new root from lane 63's R.
    __device__ __forceinline__ void replace128(uint64_t vnew, int32_t vnewI, const PathConst &pc, int lane)
    {
        const uint64_t val = readlane64(L, 63); // slot 127
        const int32_t valI = readlane32(IL, 63);
        const uint64_t lm = ballot(L > R) | (1ull << 63); // node p takes its L child (node 63: slot 127 only)
        const bool takeL = in_mask(lm);
        const uint64_t chv = takeL ? L : R;
        const int32_t chI = takeL ? IL : IR;
        const uint32_t caddr = takeL ? pc.addrL : pc.addrR;
        const uint64_t up0 = bperm64_addr(chv, caddr);
        const int32_t up0I = bperm32_addr(chI, caddr);
        const uint64_t fpre = bperm64_addr(L, pc.addrHalf);
        const int32_t fpreI = bperm32_addr(IL, pc.addrHalf);
        // keep the six fetches together: left to itself the compiler issues the father fetch after the first wait,
        // which makes two LDS round trips of the one (profiles/r04/ab_search_replace_fetch_pin.txt)
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t mv = ballot(!(val > chv));
        const uint64_t W = pc.path(mv, lm);
        // per-lane tests: the path is a chain of nodes, so its deepest node is W's highest bit
        // s_flbit of 0 is -1, so W = 0 gives 63 ^ -1 = -64: no lane and no half, no zero test needed
        uint32_t fb;
        asm("s_flbit_i32_b64 %0, %1" : "=s"(fb) : "s"(W));
        const uint32_t lastW = fb ^ 63u;
        // lane (lane >> 1) is on the path and took its L child (lane >> 1 < 32: the low word holds its bit)
        const uint32_t wlm = (uint32_t)(W & lm);
        const bool moved = (wlm >> pc.half) & 1u;
        // the single-lane writes of slot 127's value (val) are v_writelanes of the scalar, not a compare and a select
        // of a VGPR copy. Lane 0: the root after the pop -- node 0's chosen child if node 0 is on the path, else val
        // (only lane 0 is read: with node 0 on the path val goes to lane 1)
        const uint64_t rootpp = writelane64(chv, val, (uint32_t)W & 1u);
        const int32_t rootppI = writelane32(chI, valI, (uint32_t)W & 1u);
        // the chain's fathers after the pop, from the pre-pop registers (read on the chain lanes 0, 1, 3, 7, 15, 31,
        // 63 only): the moved child, or L before the pop; chain lane 2 lastW + 1 takes val when the path's end took
        // its L child (else the write goes to lane 2, off the chain); lane 0's father is the root
        // (one 64-bit bit test: the low word of W & lm, zero-extended, so a path end at lane >= 32 -- or no path --
        // tests a zero bit)
        const uint32_t kl = (((uint64_t)wlm >> (lastW & 63u)) & 1u) ? 2u * lastW + 1u : 2u;
        uint64_t fl = writelane64(moved ? chv : fpre, val, kl);
        int32_t flI = writelane32(moved ? chI : fpreI, valI, kl);
        const bool s1 = in_mask(1ull);
        fl = s1 ? rootpp : fl;
        flI = s1 ? rootppI : flI;
        // pop writes: the path nodes' chosen child slots (the path's end takes val; with no path the write to lane
        // 0 is never read), and the root
        const uint64_t up = writelane64(up0, val, lastW);
        const int32_t upI = writelane32(up0I, valI, lastW);
        const bool wl = in_mask(W & lm), wr = in_mask(W & ~lm);
        L = wl ? up : L;
        IL = wl ? upI : IL;
        R = wr ? up : R;
        IR = wr ? upI : IR;
        const bool s63 = in_mask(1ull << 63);
        const uint64_t nroot = ((uint64_t)dpp_rol1_u32(hi32(rootpp)) << 32) | dpp_rol1_u32(lo32(rootpp)); // lane 63 <- lane 0
        const int32_t nrootI = (int32_t)dpp_rol1_u32((uint32_t)rootppI);
        R = s63 ? nroot : R;
        IR = s63 ? nrootI : IR;
        // push: h = the chain's ancestors below vnew after the pop: the L halves of lanes 31, 15, 7, 3, 1, 0 (slots 63 ..
        // 1) and lane 63's R (the root, index 7)
        constexpr uint64_t kChainL = (1ull << 31) | (1ull << 15) | (1ull << 7) | (1ull << 3) | (1ull << 1) | 1ull;
        const uint32_t h = (uint32_t)__builtin_popcount((uint32_t)ballot(vnew > L) & (uint32_t)kChainL) +
                           (uint32_t)(ballot(vnew > R) >> 63); // 32-bit scalar ops: the chain's L bits are in the low word
        // index h takes vnew: chain lane (64 >> h) - 1's L (h = 7 writes lane 63's L, which the next select restores),
        // or lane 63's R (the root) when h = 7; the chain indices below h take their father's value
        L = writelane64(L, vnew, (64u >> h) - 1u);
        IL = writelane32(IL, vnewI, (64u >> h) - 1u);
        const bool sh = pc.cidx < h;
        L = sh ? fl : L;
        IL = sh ? flI : IL;
        if (h == 7u) {
            R = writelane64(R, vnew, 63u);
            IR = writelane32(IR, vnewI, 63u);
        }
    }

    // faiss heap_push(k, val) while the ef = 128 heap fills (2 <= k <= 128): val enters slot k - 1 and sifts up its
    // ancestors. Lane-mask form: each half finds its chain index (1-based position x is on the chain of k at index
    // m = bitlen(k) - bitlen(x) iff k >> m == x; lane 63's R, the root, is always on it, at index bitlen(k) - 1); the
    // ancestors below val are a bottom prefix of length h (heap order), the halves of index < h take their father's
    // value (one ds_bpermute round trip, issued first) and the half of index h takes val. No branch, no scalar
    // bookkeeping: the root is not tracked here (the caller reads it once the heap is full).
    __device__ __forceinline__ void push_fill(uint32_t k, uint64_t val, int32_t valI, const PathConst &pc)
    {
        const uint64_t fL = bperm64_addr(L, pc.addrF), fR = bperm64_addr(R, pc.addrF);
        const int32_t fIL = bperm32_addr(IL, pc.addrF), fIR = bperm32_addr(IR, pc.addrF);
        const uint32_t B = (uint32_t)bitlen(k);
        const bool s63 = in_mask(1ull << 63);
        // m < 0 (x deeper than k) wraps to a shift of 57..63: the 64-bit shift gives 0, never a position
        const uint32_t m = B - pc.bl;
        const uint32_t t = (uint32_t)((uint64_t)k >> (m & 63u));
        const uint32_t ciL = t == pc.xL ? m : 99u;
        const uint32_t ciR = s63 ? B - 1u : (t == pc.xL + 1u ? m : 99u);
        // the ancestors (index >= 1; index 0 is the new slot itself), as lane masks
        const uint64_t aL = ballot((ciL - 1u) < 7u), aR = ballot((ciR - 1u) < 7u);
        const uint32_t h = (uint32_t)(__builtin_popcountll(ballot(val > L) & aL) + __builtin_popcountll(ballot(val > R) & aR));
        const bool odd = in_mask(0xAAAAAAAAAAAAAAAAull); // father slot p odd: an L half
        const uint64_t f = odd ? fL : fR;
        const int32_t fI = odd ? fIL : fIR;
        const bool wl = ciL < h, wr = ciR < h, xl = ciL == h, xr = ciR == h;
        L = wl ? f : L;
        IL = wl ? fI : IL;
        L = xl ? val : L;
        IL = xl ? valI : IL;
        R = wr ? f : R;
        IR = wr ? fI : IR;
        R = xr ? val : R;
        IR = xr ? valI : IR;
    }
};

// bitonic sort of 128 u64 (lane l holds elements l and l + 64), ascending
__device__ __forceinline__ void sort128(uint64_t &x0, uint64_t &x1, int lane)
{
#pragma unroll
    for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride == 64) {
                // partner of element lane is element lane + 64; ascending block (size == 128)
                const uint64_t lo = x0 < x1 ? x0 : x1, hi = x0 < x1 ? x1 : x0;
                x0 = lo;
                x1 = hi;
            } else {
                const int pl = lane ^ stride;
                const uint64_t p0 = bperm64(x0, pl), p1 = bperm64(x1, pl);
                const bool lower = (lane & stride) == 0;
                const bool asc0 = (lane & size) == 0;         // element index lane
                const bool asc1 = ((lane + 64) & size) == 0;  // element index lane + 64
                const bool keepmin0 = lower == asc0, keepmin1 = lower == asc1;
                x0 = keepmin0 ? (x0 < p0 ? x0 : p0) : (x0 < p0 ? p0 : x0);
                x1 = keepmin1 ? (x1 < p1 ? x1 : p1) : (x1 < p1 ? p1 : x1);
            }
        }
    }
}

// The raw 12 bytes (id, 8-byte PQ code) of link `lane` of an inline level-0 row (DeviceIndex::rows), loaded by
// every lane (lanes past deg0 read link 0 and are masked at the use): the whole row (32 links = 384 B at
// M_hnsw = 16) is one dwordx3 load of the wave, with no branch around it, so the compiler can count it and leave
// it in flight until the next hop.
struct __attribute__((aligned(4))) Link3 {
    uint32_t x, y, z;
};
__device__ __forceinline__ Link3 load_link_raw(const int32_t *row, int lane, int deg0)
{
    return *reinterpret_cast<const Link3 *>(row + 3 * (lane < deg0 ? lane : 0));
}

// greedy_update_nearest on levels max_level .. 1 (HNSW::search, upper levels) [upstream faiss], the inline
// layout's form of greedy_upper (pq_common.h): a hop loads its upper-level list and the links' codes together
// (SearchArgs::upper_codes), one memory round trip per hop instead of two. Same distances, same order.
__device__ __forceinline__ void greedy_upper_inl(const SearchArgs &a, const float *lut, int lane, int32_t &nearest_out,
                                                 uint32_t &dn_out, int &ndis_out, int &nhops_out)
{
    int32_t nearest = a.entry_point;
    uint32_t dn = ufirst(ord32_nonneg(pq_distance_code<true>(a, lut, nearest, load_code8<true>(a, nearest))));
    int ndis = 0, nhops = 0;
    for (int level = a.max_level; level >= 1; --level) {
        const int cnt = a.cum[level + 1] - a.cum[level];
        for (;;) {
            const int32_t prev = nearest;
            const uint32_t base = a.upper_off[nearest] + (uint32_t)(a.cum[level] - a.cum[1]);
            int32_t v = -1;
            uint2 c8 = make_uint2(0u, 0u);
            if (lane < cnt) {
                v = a.upper_nbr[base + lane];
                c8 = a.upper_codes[base + lane];
            }
            const uint64_t neg = __ballot(lane < cnt && v < 0);
            const int nvalid = neg ? (__ffsll((unsigned long long)neg) - 1) : cnt;
            uint32_t dk = 0xFFFFFFFFu;
            if (lane < nvalid)
                dk = ord32_nonneg(pq_distance_code<true>(a, lut, v, c8));
            ndis += nvalid;
            nhops += 1;
            // sequential `if (dis < d_nearest)` in link order == the first lane holding the minimum: a DPP min over the
            // wave, then the lowest lane equal to it (no 64-bit shuffle reduction)
            const uint32_t mn = wave_min_u32(dk); // invalid lanes hold ~0, never below dn
            if (mn < dn) {
                dn = mn;
                nearest = __builtin_amdgcn_readlane(v, __builtin_ctzll(ballot(dk == mn)));
            }
            if (nearest == prev)
                break;
        }
    }
    nearest_out = nearest;
    dn_out = dn;
    ndis_out = ndis;
    nhops_out = nhops;
}

__device__ __forceinline__ uint64_t log_load(const uint64_t *lg, int i)
{
    return __hip_atomic_load(lg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The k (= ef) results among the log of accepted pushes: every entry with key < T, then the
// smallest (packed) ids among key == T up to k in all. T = ~0 when the heap never filled (all).
// Returns the largest packed low word admitted at key == T.
__device__ uint32_t log_id_threshold(const uint64_t *lg, int logn, uint32_t T, int k, int lane)
{
    __builtin_amdgcn_s_waitcnt(0); // this wave's log stores have landed before it reads them back
    int nlt = 0, neq = 0;
    for (int b = 0; b < logn; b += 64) {
        const int i = b + lane;
        const uint64_t e = i < logn ? log_load(lg, i) : ~0ull;
        nlt += __builtin_popcountll(ballot(i < logn && hi32(e) < T));
        neq += __builtin_popcountll(ballot(i < logn && hi32(e) == T));
    }
    const int need = k - nlt;
    if (T == 0xFFFFFFFFu || neq <= need)
        return 0xFFFFFFFFu;
    // rare: more entries at distance T than places -- binary search the need-th smallest low word
    uint32_t lo = 0u, hi = 0xFFFFFFFFu;
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        int c = 0;
        for (int b = 0; b < logn; b += 64) {
            const int i = b + lane;
            const uint64_t e = i < logn ? log_load(lg, i) : ~0ull;
            c += __builtin_popcountll(ballot(i < logn && hi32(e) == T && lo32(e) <= mid));
        }
        if (c >= need)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// Copies the selected log entries, in log order, to dst[0 .. count) and returns count (<= k).
// dst may be the log itself (in-place compaction: a block is read before any write can reach it).
template <typename Ptr>
__device__ __forceinline__ int log_select(const uint64_t *lg, int logn, uint32_t T, uint32_t idthr, Ptr dst, int lane)
{
    int cnt = 0;
    for (int b = 0; b < logn; b += 64) {
        const int i = b + lane;
        const uint64_t e = i < logn ? log_load(lg, i) : ~0ull;
        const bool sel = i < logn && (hi32(e) < T || (hi32(e) == T && lo32(e) <= idthr));
        const uint64_t sm = ballot(sel);
        if (sel)
            dst(cnt + __builtin_popcountll(sm & lanes_below(lane)), e);
        cnt += __builtin_popcountll(sm);
    }
    return cnt;
}

#ifdef DRM_PQ_TRACE
// diagnostic trace (DRM_PQ_TRACE builds, DRM_SEARCH_TRACE=1): lane 0 appends an 8-word record to host memory, which
// the host can read while the kernel runs -- or hangs
__device__ __forceinline__ void dbg_rec(const SearchArgs &a, uint32_t tag, int q, int hop, uint32_t w3, uint32_t w4, uint32_t w5,
                        uint32_t w6, uint32_t w7)
{
    if (!a.trace)
        return;
    const uint32_t i = __hip_atomic_fetch_add(a.trace, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((int64_t)i * 8 + 16 > kTraceWords)
        return;
    uint32_t *r = a.trace + 8 + (size_t)i * 8;
    const uint32_t v[8] = {tag, (uint32_t)q, (uint32_t)hop, w3, w4, w5, w6, w7};
    for (int j = 0; j < 8; ++j)
        __hip_atomic_store(r + j, v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// written by the first active lane; the tag word carries the active lane count (bits 16..23) and that lane (24..31),
// so a record made with part of the wave masked off shows it
#define DRM_DBG(tag, ...)                                                                                    \
    do {                                                                                                    \
        const uint64_t _ex = __builtin_amdgcn_read_exec();                                                  \
        if (lane == __builtin_ctzll(_ex))                                                                   \
            dbg_rec(a, (tag) | ((uint32_t)__builtin_popcountll(_ex) << 16) | ((uint32_t)lane << 24), __VA_ARGS__); \
    } while (0)
#else
#define DRM_DBG(...) do {} while (0)
#endif

#define DRM_FSTAMP(idx)                                                                                     \
    do {                                                                                                    \
        if (STAMPS) {                                                                                       \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                                               \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            st_acc[idx] += _t - st_last;                                                                    \
            st_last = _t;                                                                                   \
        }                                                                                                   \
    } while (0)

// LOGRES: k == ef (result set from the log); else k <= 64 (register result set).
// FIX128: ef = efSearch = 128 (and k = 128 with LOGRES) as compile-time constants: the pipeline's EF = K = 128,
// and the sparse default k_clusters = 5 at EF = 128 (src/main.cpp:56-63,278) -- fewer live SGPRs.
// STATS: faiss's HNSWStats.ndis (links never seen before) counted exactly with a per-slot bitmap beside the heap
// (SearchArgs::visited, cleared from a list after each query). Nothing else depends on it; without it ndis counts
// the distances the kernel computed (every valid link of every expanded row, plus the upper levels).
// STAMPS: diagnostic section timers (DRM_SEARCH_STAMPS=1).
template <bool LOGRES, bool STAMPS, bool FIX128, bool STATS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void hnsw_pq_fast_kernel(SearchArgs a)
{
    // the 8 x 256 f32 LUT (the kernel's only LDS): a static allocation at LDS address 0, so the LUT reads
    // address it with no base add
    __shared__ __align__(16) unsigned char smem[8 * 256 * sizeof(float)];
    uint64_t st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    const int lane = lane_id();
    float *lut = reinterpret_cast<float *>(smem);
    uint64_t *stage = reinterpret_cast<uint64_t *>(smem); // reuses the LUT once the walk is over
    uint32_t *vis = STATS ? a.visited + (size_t)blockIdx.x * (size_t)a.vis_words : nullptr;
    int32_t *clr = STATS ? a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap : nullptr;
    uint64_t *lg = a.log + (size_t)blockIdx.x * (size_t)a.log_cap;
    const int ef = FIX128 ? 128 : a.ef, k = (FIX128 && LOGRES) ? 128 : a.k, deg0 = a.deg0;
    const int ef_search = FIX128 ? 128 : a.efSearch;
    const int hop_bound = a.hop_bound < (int64_t)INT32_MAX ? (int)a.hop_bound : INT32_MAX;
    int64_t taken = 0;
    const PathConst pconst(lane);
    const uint32_t kInfKey = ord32(INFINITY);

    for (;;) {
        const int q = wave_next_item(a.counter, lane);
        DRM_DBG(16u, q, 0, (uint32_t)a.n, 0u, 0u, 0u, 0u);
        if ((int64_t)q >= a.n)
            break;
        if (++taken > a.item_bound) { // more items than the queue holds: a broken work-queue fetch
            if (lane == 0)
                atomicAdd(a.errors, 1u);
            break;
        }
        if (a.entry_point < 0 || a.ntotal == 0) {
            for (int j = lane; j < k; j += 64) {
                a.D[(int64_t)q * k + j] = INFINITY;
                a.I[(int64_t)q * k + j] = -1;
            }
            if (lane == 0) {
                a.ndis[q] = 0;
                a.nhops[q] = 0;
                if (a.nhops_upper)
                    a.nhops_upper[q] = 0;
            }
            continue;
        }
        DRM_FSTAMP(7);
        if (a.x_aligned16)
            build_lut_m8(a, q, lut, lane);
        else
            build_lut(a, q, lut, lane);
        DRM_FSTAMP(0);
        int32_t nearest;
        uint32_t dn;
        int ndis, nhops;
        if (a.upper_codes)
            greedy_upper_inl(a, lut, lane, nearest, dn, ndis, nhops);
        else
            greedy_upper<true>(a, lut, lane, nearest, dn, ndis, nhops);
        const int nhops_upper = nhops;
#ifdef DRM_PQ_DEBUG
        if ((nearest < 0 || nearest >= a.ntotal) && lane == 0)
            printf("[pq dbg] q %d: level-0 entry %d out of range\n", q, nearest);
#endif
        DRM_FSTAMP(1);

        // MinimaxHeap candidates(ef); candidates.push(nearest, d_nearest)
        Heap hp;
        hp.L = kUnused;
        hp.R = lane == 63 ? pack(dn, nearest) : kUnused;
        // node ids are held tagged (id ^ 2^31, the low word of their key): the pushed key's low word is the id as read,
        // no scalar XOR per push; an empty slot holds the tag of -1
        hp.IL = (int32_t)0x7FFFFFFF;
        hp.IR = lane == 63 ? (int32_t)((uint32_t)nearest ^ 0x80000000u) : (int32_t)0x7FFFFFFF;
        int kc = 1;
        // the root's key (high word) and node id, current whenever the heap is full (kc == ef): the fill does not track
        // them, they are read from lane 63's R once the heap is full, and after every full-heap replace
        uint32_t rootHi = dn;
        int32_t rootI = (int32_t)((uint32_t)nearest ^ 0x80000000u); // tagged
        // result set: the log (LOGRES) or a sorted register set of k <= 64 entries
        int logn = 0;
        uint64_t rv = ~0ull; // !LOGRES: lane j < k holds the j-th smallest (key, id) so far
        uint32_t thr = kInfKey;
        auto add_result = [&](uint64_t v) { // SingleResultHandler::add_result, k <= 64
            const int pos = __builtin_popcountll(ballot(lane < k && rv < v));
            const uint64_t sh = dpp_shr1_u64(~0ull, rv);
            rv = lane > pos ? sh : (lane == pos ? v : rv);
            thr = (uint32_t)__builtin_amdgcn_readlane((int)hi32(rv), k - 1);
        };
        // k == ef: the result set is the heap's entries (with their node ids) plus the log of evicted entries that
        // tied with the root left behind. Evictions not yet stored: lanes [0, sn) of (sbh, sbl) =
        // (key, id ^ 2^31)
        uint32_t sbh = 0u, sbl = 0u;
        int sn = 0;
        // compacts the stored log when the staged entries would overflow it -- every logged entry is at or above the
        // root, and only those at the root's distance can still be results: k of them, the smallest ids, are kept
        // (T = the root's key) -- then appends the staged entries
        auto log_compact = [&]() {
            const uint32_t T = rootHi;
            const uint32_t idthr = log_id_threshold(lg, logn, T, k, lane);
            logn = log_select(lg, logn, T, idthr, [&](int p, uint64_t e) {
                __hip_atomic_store(lg + p, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }, lane);
            __builtin_amdgcn_s_waitcnt(0);
        };
        auto log_flush = [&]() {
            if (logn + sn > a.log_cap)
                log_compact();
#ifdef DRM_PQ_DEBUG
            if (logn + sn > a.log_cap && lane == 0)
                printf("[pq dbg] q %d: log %d + %d entries past its capacity %d\n", q, logn, sn, a.log_cap);
#endif
            if (lane < sn)
                __hip_atomic_store(lg + logn + lane, ((uint64_t)sbh << 32) | sbl, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            logn += sn;
            sn = 0;
        };
        if (!LOGRES) {
            if (dn < thr)
                add_result(pack(dn, nearest));
        }
        int clear_n = 1;
        if (STATS && lane == 0) { // vt.set(entry)
            vis_test_set(&vis[nearest >> 5], 1u << (nearest & 31));
            if (a.clear_cap > 0)
                clr[0] = nearest;
        }
        DRM_DBG(1u, q, 0, (uint32_t)nearest, dn, (uint32_t)ef, (uint32_t)k, (uint32_t)ef_search);
        int nstep = 0, ndis0 = 0;
        bool overrun = false;
        int32_t pred = -1;
        // the predicted next pop_min key (the prediction's minimum): pop_min checks it with two ballots and reduces
        // over the wave only when it missed
        uint32_t dhint = 0xFFFFFFFFu;
        // a 2048-bit filter of the popped nodes (one bit per lane and word: 64 x 32), so the next-row prediction can
        // skip links back to nodes already expanded
        uint32_t popped_bits = 0u;
        Link3 praw{0xFFFFFFFFu, 0u, 0u}; // the predicted row's link `lane`, raw (pred = -1: none yet)
        // 11 bits of a 24-bit multiplicative hash (v_mul_u32_u24, full rate; a 32-bit v_mul_lo_u32 is not)
        auto pop_hash = [](int32_t v) { return (((uint32_t)v & 0xFFFFFFu) * 0x9E3779u) >> 21; };
        for (;;) {
            // every hop expands a node taken off the heap, and a node enters the heap at most once (a node in the
            // heap is seen, one that left it is at or above the root for good): more than ntotal hops means the
            // bookkeeping is broken -- end the query with an error status rather than loop
            if (nstep > hop_bound) {
                overrun = true;
                break;
            }
            // from pop_min to the issue of the next row's load the wave is on its own critical path: it runs at a
            // raised issue priority, so waves about to fetch their next row get ahead of waves in the push loop (whose
            // load is already in flight): 86.87 -> 86.45 ms at C5
            // pop_min: smallest key among valid slots, ties -> the highest slot
            const bool vL = lo32(hp.L) != kPopLo, vR = lo32(hp.R) != kPopLo;
            // MinimaxHeap::size(): the valid (filled, not popped) slots; unused slots read as popped
            const uint64_t validm = ballot(vL) | ballot(vR);
            if (validm == 0ull)
                break;
            const uint32_t cL = vL ? hi32(hp.L) : 0xFFFFFFFFu, cR = vR ? hi32(hp.R) : 0xFFFFFFFFu;
            // in-lane: slot 2l+2 (R) outranks 2l+1 (L); lane 63's R is slot 0, the lowest (a mask, not a lane value)
            const uint64_t rightm = ballot(cR < cL) | (ballot(cR == cL) & ~(1ull << 63));
            const bool pickR = in_mask(rightm);
            const uint32_t pk = pickR ? cR : cL;
            // the minimum: the hint when no slot is below it and one holds it, else a wave reduction
            uint32_t d0 = ufirst(dhint);
            uint64_t eqm = ballot(pk == d0);
            const uint64_t ltm = ballot(pk < d0);
            // one scalar test: a slot under the hint, or none at it (the compiler's own form of the two tests takes
            // seven scalar instructions)
            uint64_t bad;
            asm("s_cmp_eq_u64 %1, 0\n\ts_cselect_b64 %0, 1, 0\n\ts_or_b64 %0, %0, %2" : "=&s"(bad) : "s"(eqm), "s"(ltm) : "scc");
            if (bad != 0ull) {
                d0 = wave_min_u32(pk);
                eqm = ballot(pk == d0);
            }
            // the highest tied slot: the highest tied lane, unless that is lane 63 holding the root (slot 0)
            const uint64_t tiedm = eqm & ~(rightm & (1ull << 63));
            const int wl = tiedm ? 63 - __builtin_clzll(tiedm) : 63;
            const int32_t v0 = (int32_t)((uint32_t)__builtin_amdgcn_readlane((int)lo32(pickR ? hp.R : hp.L), wl) ^
                                         0x80000000u);
            // mark the slot popped (its id -1 in the key; IL / IR keep the node)
            const bool popR = lane == wl && pickR, popL = lane == wl && !pickR;
            hp.R = popR ? (hp.R & ~0xFFFFFFFFull) | kPopLo : hp.R;
            hp.L = popL ? (hp.L & ~0xFFFFFFFFull) | kPopLo : hp.L;
            DRM_DBG(2u, q, nstep, (uint32_t)v0, d0, (uint32_t)__builtin_popcountll(validm), (uint32_t)kc, rootHi);
            // count_below(d0): every slot in the heap (popped ones included); unused keys are ~0. The slot just popped
            // holds d0 itself, so at most ef - 1 slots lie below it: with efSearch >= ef (ef = max(efSearch, k), so
            // whenever k <= efSearch -- the pipeline's EF = K = 128) the check can never stop the search, and is skipped
            if (ef_search < ef) {
                const int below =
                    __builtin_popcountll(ballot(hi32(hp.L) < d0)) + __builtin_popcountll(ballot(hi32(hp.R) < d0));
                if (below >= ef_search)
                    break;
            }
            DRM_FSTAMP(2);

            // expand v0's level-0 row: its ids and codes arrive with one load, prefetched one hop ago when the
            // prediction held
            // from here to the issue of the next row's load the wave is on its own critical path (its current row
            // arrives, its links are scored, the next pop is predicted and fetched): it runs at a raised issue
            // priority, so waves about to fetch their next row get ahead of waves in the push loop, whose load is
            // already in flight. 86.6 -> 85.9 ms at C5; raised from pop_min on, or only from the ADC or the
            // prediction on, it gains less
            __builtin_amdgcn_s_setprio(2);
            const bool hit = v0 == pred;
            if (STAMPS) { // row prediction hits / hops
                st_acc[8] += hit ? 1u : 0u;
                st_acc[9] += 1u;
            }
            {
                const uint32_t h0 = pop_hash(v0);
                if (lane == (int)((h0 >> 5) & 63u))
                    popped_bits |= 1u << (h0 & 31u);
            }
#ifdef DRM_PQ_DEBUG
            if (v0 < 0 || v0 >= a.ntotal) {
                if (lane == 0)
                    printf("[pq dbg] q %d hop %d: v0 %d out of range (kc %d d0 %08x)\n", q, nstep, v0, kc, d0);
                overrun = true;
                break;
            }
#endif
            if (!hit)
                praw = load_link_raw(a.rows + (size_t)v0 * (size_t)a.row_words, lane, deg0);
            const int32_t v1 = lane < deg0 ? (int32_t)praw.x : -1;
            const uint2 c8 = make_uint2(praw.y, praw.z); // past deg0: link 0's code (the LUT reads stay in the LUT)
            const int32_t v1x = (int32_t)((uint32_t)v1 ^ 0x80000000u); // the links' ids tagged, as the heap holds them
            const uint64_t negm = ballot(v1 < 0);
            const int jmax = negm ? __builtin_ctzll(negm) : 64; // lanes past deg0 hold -1
            const uint64_t actm = negm ? (negm & (0ull - negm)) - 1ull : ~0ull;
            DRM_FSTAMP(10);
            if (STAMPS) { // the 128-B lines the row's valid links span (10, 21, 32 links per 1, 2, 3 lines)
                st_acc[12] += jmax <= 10 ? 1u : 0u;
                st_acc[13] += (jmax > 10 && jmax <= 21) ? 1u : 0u;
                st_acc[14] += jmax > 21 ? 1u : 0u;
            }
            DRM_DBG(3u, q, nstep, (uint32_t)jmax, (uint32_t)pred, (uint32_t)hit, (uint32_t)__builtin_amdgcn_readfirstlane(v1),
                    (uint32_t)logn);
            // PQ-ADC distance of every link (the codes came with the row), then the predicted next pop_min: the
            // smallest valid heap slot or link not known to be popped; its row is fetched now and waited for at
            // the next hop
            const uint32_t dall = adc8(lut, c8);
            {
                const uint32_t hv = pop_hash(v1);
                const uint32_t pw = bperm32(popped_bits, (int)((hv >> 5) & 63u));
                const bool known_popped = (pw >> (hv & 31u)) & 1u;
                const uint32_t dp = (lane < jmax && !known_popped) ? dall : 0xFFFFFFFFu;
                // the valid slots' keys: pop_min's, less the slot it just popped
                const uint32_t hL = popL ? 0xFFFFFFFFu : cL;
                const uint32_t hR = popR ? 0xFFFFFFFFu : cR;
                // one v_min3 (the compiler folds popR's select past the first min and then needs two mins + a select)
                uint32_t mk;
                asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mk) : "v"(dp), "v"(hL), "v"(hR));
                const int32_t hid = hL == mk ? unpack_id(hp.L) : unpack_id(hp.R);
                const int32_t mid = dp == mk ? v1 : hid;
                const uint32_t mm = wave_min_u32(mk);
                dhint = mm;
                pred = -1;
                // no prediction (the heap and the row hold nothing valid): load v0's row again, pred stays -1
                int32_t pnode = v0;
                if (mm != 0xFFFFFFFFu) {
                    pred = __builtin_amdgcn_readlane(mid, __builtin_ctzll(ballot(mk == mm)));
                    pnode = pred;
                }
#ifdef DRM_PQ_DEBUG
                if (pnode < 0 || pnode >= a.ntotal) {
                    if (lane == 0)
                        printf("[pq dbg] q %d hop %d: predicted node %d out of range (mm %08x)\n", q, nstep, pnode, mm);
                    pnode = v0;
                }
#endif
                praw = load_link_raw(a.rows + (size_t)pnode * (size_t)a.row_words, lane, deg0);
                __builtin_amdgcn_s_setprio(0);
            }
            if (STATS) {
                // VisitedTable get + set of every link, in row order (lanes of one atomic instruction that share a
                // word are serialised: exactly one finds a repeated id fresh); the count is all it feeds
                const bool act = lane < jmax;
                const uint32_t bit = 1u << (v1 & 31);
                const uint32_t old = act ? vis_test_set(&vis[v1 >> 5], bit) : 0xFFFFFFFFu;
                const bool fresh = act && !(old & bit);
                const uint64_t fm = ballot(fresh);
                if (fresh) { // VisitedTable::advance list
                    const int p = clear_n + __builtin_popcountll(fm & lanes_below(lane));
                    if (p < a.clear_cap)
                        clr[p] = v1;
                }
                clear_n += __builtin_popcountll(fm);
                ndis0 += __builtin_popcountll(fm);
            } else {
                ndis0 += jmax;
            }
            DRM_FSTAMP(3);
            // add_to_heap for each link not seen before, in row order. On a full heap a link at or above the root is
            // rejected now and on any later encounter (the root only falls): skipped whether seen or not. A link
            // below the root was seen iff it is in the heap (popped or not): a seen link either entered the heap
            // and is still there, or was rejected / evicted at a root that is now at or below its distance.
            uint64_t rem = actm;
            if (__builtin_expect(kc < ef, 0)) { // the heap fills: every link not in it is pushed
                while (rem) {
                    const int l = __builtin_ctzll(rem);
                    asm("s_bitset0_b64 %0, %1" : "+s"(rem) : "s"(l)); // rem &= rem - 1, one scalar op
                    const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)dall, l);
                    const int32_t idl = __builtin_amdgcn_readlane(v1x, l); // tagged
                    if (STAMPS)
                        st_acc[4] += 1u; // links tested against the heap's ids
                    if (hp.holds(idl))
                        continue;
                    const uint64_t val = ((uint64_t)key << 32) | (uint32_t)idl;
                    DRM_DBG(4u, q, nstep, (uint32_t)idl, key, (uint32_t)kc, 0u, (uint32_t)sn);
                    if (!LOGRES && key < thr)
                        add_result(val);
                    ++kc;
                    if (ef == 128)
                        hp.push_fill((uint32_t)kc, val, idl, pconst);
                    else
                        hp.push(kc, val, idl, lane);
                    if (kc == ef) { // full: the root is read once, and kept current from here on
                        rootHi = hp.root_hi();
                        rootI = hp.root_id();
                        break;
                    }
                }
            }
            rem &= ballot(dall < rootHi); // the heap is full here, or rem is empty
            while (rem) { // MinimaxHeap::push on the full heap: pop the max, push val
                const int l = __builtin_ctzll(rem);
                asm("s_bitset0_b64 %0, %1" : "+s"(rem) : "s"(l)); // rem &= rem - 1, one scalar op
                const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)dall, l);
                const int32_t idl = __builtin_amdgcn_readlane(v1x, l); // tagged
                if (STAMPS)
                    st_acc[4] += 1u;
                if (hp.holds(idl))
                    continue;
                const uint64_t val = ((uint64_t)key << 32) | (uint32_t)idl;
                DRM_DBG(4u, q, nstep, (uint32_t)idl, key, (uint32_t)kc, 0u, (uint32_t)sn);
                if (!LOGRES && key < thr)
                    add_result(val);
                const uint32_t evk = rootHi; // the evicted slot: the root (its node id in rootI)
                const int32_t evi = rootI;
                if (ef == 128) {
                    hp.replace128(val, idl, pconst, lane);
                    if (STAMPS)
                        st_acc[11] += 1u;
                } else {
                    hp.pop(kc, lane);
                    hp.push(kc, val, idl, lane);
                }
                rootHi = hp.root_hi();
                rootI = hp.root_id();
                // the root fell: links at or above it leave the candidate mask (one compare for the rest of the row)
                rem &= ballot(dall < rootHi);
                // LOGRES: an evicted result at the new root's distance can still be among the k results (the result
                // handler breaks distance ties by node id, the MinimaxHeap by slot); any other evicted one cannot
                if (LOGRES && evk == rootHi) {
                    if (sn == 64)
                        log_flush();
                    const bool at = lane == sn; // lane sn takes the entry (one compare, two selects)
                    sbh = at ? evk : sbh;
                    sbl = at ? (uint32_t)evi : sbl; // already tagged
                    ++sn;
                }
            }
            nstep++;
            DRM_FSTAMP(5);
        }
        __builtin_amdgcn_s_setprio(0); // the loop's exits leave from the raised section
        DRM_FSTAMP(2);

        // --- SingleResultHandler::end (heap_reorder): ascending (distance, id), (+inf, -1) padding
        DRM_DBG(6u, q, nstep, (uint32_t)(uintptr_t)lg, (uint32_t)((uintptr_t)lg >> 32), (uint32_t)a.log_cap,
                (uint32_t)sn, (uint32_t)logn);
        if (LOGRES) {
            if (sn)
                log_flush();
            // the heap's entries join the log, with their node ids (slots never filled are left out); room for them:
            // a compacted log holds at most k entries, and log_cap >= k + ef (host side)
            if (logn + kc > a.log_cap)
                log_compact();
            {
                const bool hl = hp.IL != (int32_t)0x7FFFFFFF, hr = hp.IR != (int32_t)0x7FFFFFFF; // filled slots
                const uint64_t mL = ballot(hl), mR = ballot(hr), below = lanes_below(lane);
                if (hl)
                    __hip_atomic_store(lg + logn + __builtin_popcountll(mL & below), ((uint64_t)hi32(hp.L) << 32) | (uint32_t)hp.IL,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (hr)
                    __hip_atomic_store(lg + logn + __builtin_popcountll(mL) + __builtin_popcountll(mR & below),
                                       ((uint64_t)hi32(hp.R) << 32) | (uint32_t)hp.IR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef DRM_PQ_DEBUG
                if (__builtin_popcountll(mL) + __builtin_popcountll(mR) != kc && lane == 0)
                    printf("[pq dbg] q %d: %d heap slots hold an id, %d filled\n", q,
                           __builtin_popcountll(mL) + __builtin_popcountll(mR), kc);
#endif
                logn += __builtin_popcountll(mL) + __builtin_popcountll(mR);
            }
            DRM_DBG(7u, q, nstep, (uint32_t)logn, 0u, 0u, 0u, 0u);
            __builtin_amdgcn_s_waitcnt(0); // this wave's log stores have landed
            DRM_DBG(8u, q, nstep, 0u, 0u, 0u, 0u, 0u);
            __syncthreads();
            const uint32_t T = kc == ef ? rootHi : 0xFFFFFFFFu;
            const uint32_t idthr = log_id_threshold(lg, logn, T, k, lane);
            DRM_DBG(9u, q, nstep, T, idthr, 0u, 0u, 0u);
            const int c = log_select(lg, logn, T, idthr, [&](int p, uint64_t e) { stage[p] = e; }, lane);
            DRM_DBG(10u, q, nstep, (uint32_t)c, 0u, 0u, 0u, 0u);
#ifdef DRM_PQ_DEBUG
            if (c > k && lane == 0)
                printf("[pq dbg] q %d: %d results selected from a log of %d (T %08x)\n", q, c, logn, T);
#endif
            __syncthreads();
            DRM_DBG(11u, q, nstep, 0u, 0u, 0u, 0u, 0u);
            {
                uint64_t x0 = lane < c ? stage[lane] : ~0ull;
                uint64_t x1 = lane + 64 < c ? stage[lane + 64] : ~0ull;
                sort128(x0, x1, lane);
                DRM_DBG(12u, q, nstep, 0u, 0u, 0u, 0u, 0u);
                __syncthreads();
                stage[lane] = x0;
                stage[lane + 64] = x1;
                __syncthreads();
            }
            DRM_DBG(13u, q, nstep, (uint32_t)(uintptr_t)a.D, (uint32_t)((uintptr_t)a.D >> 32), (uint32_t)(uintptr_t)a.I,
                    (uint32_t)((uintptr_t)a.I >> 32), (uint32_t)k);
            for (int j = lane; j < k; j += 64) {
                const int64_t o = (int64_t)q * k + j;
                const uint64_t e = stage[j];
                a.D[o] = j < c ? unord32(hi32(e)) : INFINITY;
                a.I[o] = j < c ? (int64_t)unpack_id(e) : (int64_t)-1;
            }
            DRM_DBG(14u, q, nstep, 0u, 0u, 0u, 0u, 0u);
            __syncthreads();
            DRM_DBG(15u, q, nstep, 0u, 0u, 0u, 0u, 0u);
        } else if (lane < k) {
            const int64_t o = (int64_t)q * k + lane;
            const bool valid = rv != ~0ull;
            a.D[o] = valid ? unord32(hi32(rv)) : INFINITY;
            a.I[o] = valid ? (int64_t)unpack_id(rv) : (int64_t)-1;
        }
        DRM_DBG(5u, q, nstep, (uint32_t)logn, (uint32_t)overrun, (uint32_t)kc, rootHi, 0u);
        if (lane == 0) {
            a.ndis[q] = overrun ? -1 : ndis + ndis0;
            a.nhops[q] = overrun ? -1 : nhops + nstep;
            if (a.nhops_upper)
                a.nhops_upper[q] = nhops_upper;
            if (overrun)
                atomicAdd(a.errors, 1u);
        }
        DRM_DBG(18u, q, nstep, 0u, 0u, 0u, 0u, 0u);
        if (STATS) { // VisitedTable::advance: clear exactly the bits this query set; they land before the next query
            if (clear_n <= a.clear_cap) {
                for (int t = lane; t < clear_n; t += 64)
                    vis[clr[t] >> 5] = 0u;
            } else {
                for (int64_t w = lane; w < a.vis_words; w += 64)
                    vis[w] = 0u;
            }
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        }
        DRM_FSTAMP(6);
    }
    DRM_DBG(17u, 0, 0, 0u, 0u, 0u, 0u, 0u);
    if (STAMPS && lane == 0 && a.stamps)
        for (int i = 0; i < 16; ++i)
            atomicAdd(reinterpret_cast<unsigned long long *>(a.stamps) + i, (unsigned long long)st_acc[i]);
}

// DeviceIndex::rows: row i holds, for each link j < deg0, its id then its 8-byte code at words [3j, 3j + 3) (code 0
// past the row's end). One wave per node; lane j < deg0 writes link j.
__global__ __launch_bounds__(256) void build_inline_rows_kernel(const int32_t *nbr0, const uint8_t *codes, int64_t n,
                                                                int deg0, int row_words, int32_t *rows)
{
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int j = threadIdx.x & 63;
    if (i >= n || j >= deg0)
        return;
    const int32_t v = nbr0[i * deg0 + j];
    int32_t *e = rows + i * (int64_t)row_words + 3 * j;
    const uint2 c = v >= 0 ? *reinterpret_cast<const uint2 *>(codes + (size_t)v * 8) : make_uint2(0u, 0u);
    e[0] = v;
    e[1] = (int32_t)c.x;
    e[2] = (int32_t)c.y;
}

__global__ __launch_bounds__(256) void build_upper_codes_kernel(const int32_t *upper_nbr, const uint8_t *codes, int64_t n,
                                                                uint2 *out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const int32_t v = upper_nbr[i];
    out[i] = v >= 0 ? *reinterpret_cast<const uint2 *>(codes + (size_t)v * 8) : make_uint2(0u, 0u);
}

} // namespace

void build_inline_rows(DeviceIndex &ix)
{
    if (ix.pq_M != 8 || ix.pq_nbits != 8 || ix.code_size != 8 || ix.deg0 > 64 || ix.deg0 < 1 ||
        ix.ntotal <= 0)
        return;
    const int64_t words = ((int64_t)ix.deg0 * 3 + 31) / 32 * 32; // deg0 x (id, 2 code words), 128-B rows
    DRM_HIP_CHECK(malloc_big((void **)&ix.rows, sizeof(int32_t) * (size_t)ix.ntotal * (size_t)words, kBigIndex));
    ix.row_words = (int32_t)words;
    ix.device_bytes += (int64_t)sizeof(int32_t) * ix.ntotal * words;
    const int64_t blocks = (ix.ntotal + 3) / 4;
    for (int64_t b0 = 0; b0 < blocks; b0 += (int64_t)1 << 30) {
        const int64_t nb = std::min<int64_t>(blocks - b0, (int64_t)1 << 30);
        hipLaunchKernelGGL(build_inline_rows_kernel, dim3((unsigned)nb), dim3(256), 0, 0, ix.nbr0 + b0 * 4 * ix.deg0,
                           ix.codes, std::min<int64_t>(ix.ntotal - b0 * 4, nb * 4), ix.deg0, (int)words,
                           ix.rows + b0 * 4 * words);
        DRM_HIP_CHECK(hipGetLastError());
    }
    if (ix.upper_len > 0) {
        DRM_HIP_CHECK(malloc_big((void **)&ix.upper_codes, sizeof(uint2) * (size_t)ix.upper_len, kBigIndex));
        ix.device_bytes += (int64_t)sizeof(uint2) * ix.upper_len;
        const int64_t ub = (ix.upper_len + 255) / 256;
        for (int64_t b0 = 0; b0 < ub; b0 += (int64_t)1 << 30) {
            const int64_t nb = std::min<int64_t>(ub - b0, (int64_t)1 << 30);
            hipLaunchKernelGGL(build_upper_codes_kernel, dim3((unsigned)nb), dim3(256), 0, 0, ix.upper_nbr + b0 * 256,
                               ix.codes, std::min<int64_t>(ix.upper_len - b0 * 256, nb * 256), ix.upper_codes + b0 * 256);
            DRM_HIP_CHECK(hipGetLastError());
        }
    }
    DRM_HIP_CHECK(hipDeviceSynchronize());
}

bool hnsw_pq_fast_supported(const DeviceIndex &ix, int k, int efc)
{
    return ix.rows != nullptr && ix.pq_M == 8 && ix.pq_nbits == 8 && ix.code_size == 8 && ix.deg0 <= 64 &&
           efc <= 128 && (k == efc || k <= 64);
}

void launch_hnsw_pq_fast(const SearchArgs &a, int slots, bool stamps, hipStream_t stream)
{
    const bool logres = a.k == a.ef;
    const bool fix = a.ef == 128 && a.efSearch == 128;
    const bool stats = a.exact_stats != 0;
#define DRM_LAUNCH_FAST(LR, ST, FX, XS)                                                                          \
    hipLaunchKernelGGL((hnsw_pq_fast_kernel<LR, ST, FX, XS>), dim3(slots), dim3(64), 0, stream, a)
    if (stamps && logres && fix && !stats)
        DRM_LAUNCH_FAST(true, true, true, false);
    else if (stats) {
        if (fix && logres)
            DRM_LAUNCH_FAST(true, false, true, true);
        else if (fix)
            DRM_LAUNCH_FAST(false, false, true, true);
        else if (logres)
            DRM_LAUNCH_FAST(true, false, false, true);
        else
            DRM_LAUNCH_FAST(false, false, false, true);
    } else if (fix && logres)
        DRM_LAUNCH_FAST(true, false, true, false);
    else if (fix)
        DRM_LAUNCH_FAST(false, false, true, false);
    else if (logres)
        DRM_LAUNCH_FAST(true, false, false, false);
    else
        DRM_LAUNCH_FAST(false, false, false, false);
#undef DRM_LAUNCH_FAST
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
