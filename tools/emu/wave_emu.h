// tools/emu/wave_emu.h -- host emulation of the lean search kernel's wave-parallel MinimaxHeap with node ids
// (deepreadmapper_amd/csrc/hnsw_pq_fast.hip, struct Heap and PathConst): each VGPR is an array of 64 lanes;
// ballot, readlane, ds_bpermute and inverse_ballot are loops. Test infrastructure for tools/emu/*.cpp.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using u64 = uint64_t;
using u32 = uint32_t;
constexpr int W = 64;
constexpr u32 kPopLo = 0x7FFFFFFFu;
constexpr u64 kUnused = 0xFFFFFFFF7FFFFFFFull;
template <class T> struct V { T v[W]; };
static u64 ballot(const bool *p) { u64 m = 0; for (int l = 0; l < W; ++l) if (p[l]) m |= 1ull << l; return m; }
static int bitlen(u32 x) { return 32 - __builtin_clz(x); }
static u64 pack(u32 key, int32_t id) { return ((u64)key << 32) | (u32)((u32)id ^ 0x80000000u); }
static u32 hi32(u64 v) { return (u32)(v >> 32); }
static u32 lo32(u64 v) { return (u32)v; }
static bool sgt64(u64 a, u64 b) { return a > b; }

struct PathConst {
    // lane p holds the children of node p: slot 2p+1 (L, 1-based position 2p+2) and slot 2p+2 (R, 2p+3); lane 63's R
    // is the root (1-based position 1). xL / xR / blL / blR: those positions and their bit lengths; addrF: the lane
    // holding this lane's father slot p (its L half when p is odd, its R half when p is even; lane 63's R for p = 0)
    u32 Alo[W], Ahi[W], Auplo[W], Lreqlo[W], addrL[W], addrR[W], addrHalf[W], xL[W], xR[W], blL[W], blR[W], addrF[W];
    // replace128: the chain index of each half on slot 127's ancestor chain (127 = 0, 63 = 1, ..., 1 = 6, the root 7;
    // 15 = not on it)
    u32 cidxL[W], cidxR[W];
    PathConst() {
        for (int lane = 0; lane < W; ++lane) {
            addrL[lane] = (u32)((2 * lane + 1) & 63); addrR[lane] = (u32)((2 * lane + 2) & 63);
            addrHalf[lane] = (u32)(lane >> 1);
            xL[lane] = 2u * lane + 2u; blL[lane] = bitlen(2u * lane + 2u);
            xR[lane] = lane == 63 ? 1u : 2u * lane + 3u; blR[lane] = lane == 63 ? 1u : blL[lane];
            addrF[lane] = lane > 0 ? (u32)((lane - 1) >> 1) : 63u;
            cidxL[lane] = ((lane + 1) & lane) == 0 ? 6u - (u32)(31 - __builtin_clz((u32)lane + 1u)) : 15u;
            cidxR[lane] = lane == 63 ? 7u : 15u;
            u64 A = 1ull << lane, Aup = 0, Lreq = 0;
            for (int c = lane; c > 0;) { int a = (c - 1) >> 1; A |= 1ull << a; Aup |= 1ull << a; if (c & 1) Lreq |= 1ull << a; c = a; }
            Alo[lane] = (u32)A; Ahi[lane] = (u32)(A >> 32); Auplo[lane] = (u32)Aup; Lreqlo[lane] = (u32)Lreq;
        }
    }
    // the lanes on the sift-down path: p and all its ancestors have mv set, and every ancestor chose the child toward
    // p (lm: the nodes that take their L child) -- one per-lane test, one ballot
    u64 path(u64 mv, u64 lm) const {
        bool p[W];
        for (int l = 0; l < W; ++l)
            p[l] = ((~(u32)mv & Alo[l]) | (((u32)lm ^ Lreqlo[l]) & Auplo[l]) | (~(u32)(mv >> 32) & Ahi[l])) == 0u;
        return ballot(p);
    }
};

struct Heap {
    u64 L[W], R[W];
    int32_t IL[W], IR[W];
    bool holds(int32_t v) const { for (int l = 0; l < W; ++l) if (IL[l] == v || IR[l] == v) return true; return false; }
    // Heap::replace128 (lane-mask form, the root's bookkeeping in lane 63's R): returns the new root's key
    u64 replace128(u64 vnew, int32_t vnewI, const PathConst &pc, int32_t &rootI) {
        const u64 val = L[63]; const int32_t valI = IL[63];
        bool t[W];
        for (int l = 0; l < W; ++l) t[l] = L[l] > R[l];
        const u64 lm = ballot(t) | (1ull << 63);
        u64 chv[W]; int32_t chI[W]; u32 caddr[W];
        for (int l = 0; l < W; ++l) { bool tl = (lm >> l) & 1; chv[l] = tl ? L[l] : R[l]; chI[l] = tl ? IL[l] : IR[l]; caddr[l] = tl ? pc.addrL[l] : pc.addrR[l]; }
        u64 up0[W], fpre[W]; int32_t up0I[W], fpreI[W];
        for (int l = 0; l < W; ++l) { up0[l] = chv[caddr[l]]; up0I[l] = chI[caddr[l]]; fpre[l] = L[pc.addrHalf[l]]; fpreI[l] = IL[pc.addrHalf[l]]; }
        for (int l = 0; l < W; ++l) t[l] = !(val > chv[l]);
        const u64 mv = ballot(t);
        const u64 Wm = pc.path(mv, lm);
        const u64 wlm = Wm & lm;
        u64 fl[W]; int32_t flI[W];
        // lane 0: the root after the pop (node 0's chosen child if node 0 is on the path); lane 63 takes it (DPP rotate)
        const bool on0 = (Wm & 1ull) != 0ull;
        const u64 rootpp = on0 ? chv[0] : val; const int32_t rootppI = on0 ? chI[0] : valI;
        for (int l = 0; l < W; ++l) {
            const u32 half = (u32)l >> 1;
            const bool atlast = (Wm >> l) == 1ull, klast = (Wm >> half) == 1ull, moved = ((wlm >> half) & 1ull) != 0ull;
            fl[l] = moved ? (klast ? val : chv[l]) : fpre[l]; flI[l] = moved ? (klast ? valI : chI[l]) : fpreI[l];
            if (l == 0) { fl[l] = rootpp; flI[l] = rootppI; } // the chain's top father: the root
            const u64 up = atlast ? val : up0[l]; const int32_t upI = atlast ? valI : up0I[l];
            if ((wlm >> l) & 1) { L[l] = up; IL[l] = upI; }
            if (((Wm & ~lm) >> l) & 1) { R[l] = up; IR[l] = upI; }
        }
        R[63] = rootpp; IR[63] = rootppI;
        for (int l = 0; l < W; ++l) t[l] = vnew > (pc.cidxR[l] == 7u ? R[l] : (pc.cidxL[l] != 15u ? L[l] : ~0ull));
        const u32 h = (u32)__builtin_popcountll(ballot(t));
        for (int l = 0; l < W; ++l) {
            if (pc.cidxL[l] < h) { L[l] = fl[l]; IL[l] = flI[l]; }
            if (pc.cidxL[l] == h) { L[l] = vnew; IL[l] = vnewI; }
            if (pc.cidxR[l] == h) { R[l] = vnew; IR[l] = vnewI; }
        }
        rootI = IR[63];
        return R[63];
    }
    // heap_push(k, val) while the ef = 128 heap fills (2 <= k <= 128), lane-mask form: each half finds its chain
    // index (1-based position x is on the chain of k at index m iff k >> m == x, m = bitlen(k) - bitlen(x)), the
    // ancestors below val are a bottom prefix of length h, the halves of index < h take their father's value and the
    // half of index h takes val. The root (lane 63's R) is the chain's last index. The root is not tracked here.
    void push_fill(int k, u64 val, int32_t valI, const PathConst &pc) {
        const u32 B = (u32)bitlen((u32)k);
        u64 f[W]; int32_t fI[W]; u32 ciL[W], ciR[W];
        bool a1[W], a2[W];
        for (int l = 0; l < W; ++l) {
            const u32 s = pc.addrF[l]; const bool odd = l & 1;
            f[l] = odd ? L[s] : R[s]; fI[l] = odd ? IL[s] : IR[s];
            const u32 mL = B - pc.blL[l], mR = B - pc.blR[l]; // wraps when negative: the 64-bit shift then gives 0
            const u64 tL = (u64)(u32)k >> (mL & 63u), tR = (u64)(u32)k >> (mR & 63u);
            ciL[l] = tL == pc.xL[l] ? mL : 99u; ciR[l] = tR == pc.xR[l] ? mR : 99u;
            a1[l] = val > ((ciL[l] - 1u) < 7u ? L[l] : ~0ull);
            a2[l] = val > ((ciR[l] - 1u) < 7u ? R[l] : ~0ull);
        }
        const u32 h = (u32)(__builtin_popcountll(ballot(a1)) + __builtin_popcountll(ballot(a2)));
        for (int l = 0; l < W; ++l) {
            if (ciL[l] < h) { L[l] = f[l]; IL[l] = fI[l]; }
            if (ciL[l] == h) { L[l] = val; IL[l] = valI; }
            if (ciR[l] < h) { R[l] = f[l]; IR[l] = fI[l]; }
            if (ciR[l] == h) { R[l] = val; IR[l] = valI; }
        }
    }
    // general heap_pop(k) / heap_push(k, val) (ef < 128): Heap::pop / Heap::push of the kernel, lane by lane
    u64 get(int s) const { if (s == 0) return R[63]; int o = (s - 1) >> 1; return (s & 1) ? L[o] : R[o]; }
    int32_t get_id(int s) const { if (s == 0) return IR[63]; int o = (s - 1) >> 1; return (s & 1) ? IL[o] : IR[o]; }
    void pop(int k) {
        const u64 val = get(k - 1); const int32_t valI = get_id(k - 1);
        bool takeL[W], moves[W]; int ch[W], n[W]; u64 chv[W]; int32_t chI[W];
        for (int lane = 0; lane < W; ++lane) {
            const bool has_l = 2 * lane + 1 <= k - 1, has_r = 2 * lane + 2 <= k - 1 && lane != 63;
            takeL[lane] = !has_r || L[lane] > R[lane];
            ch[lane] = takeL[lane] ? 2 * lane + 1 : 2 * lane + 2;
            chv[lane] = takeL[lane] ? L[lane] : R[lane]; chI[lane] = takeL[lane] ? IL[lane] : IR[lane];
            moves[lane] = has_l && !(val > chv[lane]);
            n[lane] = moves[lane] ? ch[lane] : lane;
        }
        for (int r = 0; r < 3; ++r) { int t[W]; for (int l = 0; l < W; ++l) t[l] = n[n[l] & 63]; for (int l = 0; l < W; ++l) n[l] = n[l] < 64 ? t[l] : n[l]; }
        const int hole = n[0];
        u64 up[W]; int32_t upI[W];
        for (int l = 0; l < W; ++l) { up[l] = chv[ch[l] & 63]; upI[l] = chI[ch[l] & 63]; }
        const u64 rootv = hole != 0 ? chv[0] : val; const int32_t rootI = hole != 0 ? chI[0] : valI;
        for (int lane = 0; lane < W; ++lane) {
            const uint32_t hx = (uint32_t)hole + 1u;
            const int sh = bitlen(hx) - bitlen((uint32_t)lane + 1u);
            const bool writer = sh > 0 && (hx >> sh) == (uint32_t)lane + 1u;
            const bool at_hole = ch[lane] == hole;
            const u64 nv = at_hole ? val : up[lane]; const int32_t nvI = at_hole ? valI : upI[lane];
            if (writer && takeL[lane]) { L[lane] = nv; IL[lane] = nvI; }
            if (writer && !takeL[lane]) { R[lane] = nv; IR[lane] = nvI; }
        }
        R[63] = rootv; IR[63] = rootI;
    }
    void push(int k, u64 val, int32_t valI) {
        u64 av[W]; int32_t avI[W]; bool moves[W];
        for (int lane = 0; lane < W; ++lane) {
            const int aj = (lane >= 1 && lane < 8) ? (k >> lane) : 0;
            const int t = aj - 1; const int owner = t <= 0 ? 63 : (t - 1) >> 1; const bool sideR = t <= 0 || !(t & 1);
            av[lane] = sideR ? R[owner] : L[owner]; avI[lane] = sideR ? IR[owner] : IL[owner];
            moves[lane] = aj >= 1 && val > av[lane];
        }
        const int h = __builtin_popcountll(ballot(moves));
        const int bk = bitlen((uint32_t)k);
        u64 nL[W], nR[W]; int32_t nIL[W], nIR[W];
        for (int lane = 0; lane < W; ++lane) {
            nL[lane] = L[lane]; nR[lane] = R[lane]; nIL[lane] = IL[lane]; nIR[lane] = IR[lane];
            const uint32_t xl = 2u * (uint32_t)lane + 2u, xr = xl + 1u;
            const int ml = bk - bitlen(xl), mr = bk - bitlen(xr);
            const bool onL = ml >= 0 && ml <= h && (uint32_t)(k >> ml) == xl;
            const bool onR = lane != 63 && mr >= 0 && mr <= h && (uint32_t)(k >> mr) == xr;
            const int m = onL ? ml : mr;
            const u64 pulled = av[(m + 1) & 63]; const int32_t pulledI = avI[(m + 1) & 63];
            const u64 nv = (m == h) ? val : pulled; const int32_t nvI = (m == h) ? valI : pulledI;
            if (onL) { nL[lane] = nv; nIL[lane] = nvI; }
            if (onR) { nR[lane] = nv; nIR[lane] = nvI; }
        }
        for (int lane = 0; lane < W; ++lane) { L[lane] = nL[lane]; R[lane] = nR[lane]; IL[lane] = nIL[lane]; IR[lane] = nIR[lane]; }
        if (h == bk - 1) { R[63] = val; IR[63] = valI; }
    }
};


