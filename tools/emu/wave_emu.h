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
    u32 Alo[W], Auplo[W], Lreqlo[W], addrL[W], addrR[W], addrHalf[W], c2[W], bl[W], addrF[W];
    PathConst() {
        for (int lane = 0; lane < W; ++lane) {
            addrL[lane] = (u32)((2 * lane + 1) & 63); addrR[lane] = (u32)((2 * lane + 2) & 63);
            addrHalf[lane] = (u32)(lane >> 1); c2[lane] = 2u * lane + 2u; bl[lane] = bitlen(2u * lane + 2u);
            addrF[lane] = lane > 0 ? (u32)((lane - 1) >> 1) : 0u;
            u64 A = 1ull << lane, Aup = 0, Lreq = 0;
            for (int c = lane; c > 0;) { int a = (c - 1) >> 1; A |= 1ull << a; Aup |= 1ull << a; if (c & 1) Lreq |= 1ull << a; c = a; }
            Alo[lane] = (u32)A; Auplo[lane] = (u32)Aup; Lreqlo[lane] = (u32)Lreq;
        }
    }
    u64 path(u64 mv, u64 lm) const {
        bool p1[W], p2[W];
        for (int l = 0; l < W; ++l) { p1[l] = ((u32)mv & Alo[l]) == Alo[l]; p2[l] = ((u32)lm & Auplo[l]) == Lreqlo[l]; }
        return ballot(p1) & (mv | 0xFFFFFFFFull) & ballot(p2);
    }
};

struct Heap {
    u64 L[W], R[W];
    int32_t IL[W], IR[W];
    bool holds(int32_t v) const { for (int l = 0; l < W; ++l) if (IL[l] == v || IR[l] == v) return true; return false; }
    // Heap::replace128, straight-line (every case a lane mask; lane 63's R / IR hold the root on return)
    u64 replace128(u64 vnew, int32_t vnewI, const PathConst &pc, int32_t &rootI) {
        constexpr u64 kHold = (1ull << 63) | (1ull << 31) | (1ull << 15) | (1ull << 7) | (1ull << 3) | (1ull << 1) | 1ull;
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
        const int last = 63 - __builtin_clzll(Wm | 1ull);
        const bool r0 = (Wm & 1ull) != 0ull;
        const u64 rootv = r0 ? chv[0] : val; const int32_t rI = r0 ? chI[0] : valI;
        const u64 wlm = Wm & lm, wrm = Wm & ~lm;
        u64 fl[W]; int32_t flI[W];
        for (int l = 0; l < W; ++l) {
            const u32 half = (u32)l >> 1;
            const bool moved = (((u32)wlm >> half) & 1u) != 0u, klast = half == (u32)last;
            fl[l] = moved ? (klast ? val : chv[l]) : fpre[l]; flI[l] = moved ? (klast ? valI : chI[l]) : fpreI[l];
            const bool atlast = l == last;
            const u64 up = atlast ? val : up0[l]; const int32_t upI = atlast ? valI : up0I[l];
            if ((wlm >> l) & 1) { L[l] = up; IL[l] = upI; }
            if ((wrm >> l) & 1) { R[l] = up; IR[l] = upI; }
        }
        for (int l = 0; l < W; ++l) t[l] = vnew > (l == 63 ? rootv : L[l]);
        const int h = __builtin_popcountll(ballot(t) & kHold);
        fl[0] = rootv; flI[0] = rI;
        const u64 shm = h ? kHold & (~0ull << ((1u << (7 - h)) - 1u)) : 0ull;
        const u64 xm = h < 7 ? 1ull << ((1u << (6 - h)) - 1u) : 0ull;
        for (int l = 0; l < W; ++l) {
            if ((shm >> l) & 1) { L[l] = fl[l]; IL[l] = flI[l]; }
            if ((xm >> l) & 1) { L[l] = vnew; IL[l] = vnewI; }
        }
        const u64 nroot = h == 7 ? vnew : rootv;
        rootI = h == 7 ? vnewI : rI;
        R[63] = nroot; IR[63] = rootI;
        return nroot;
    }
    u64 push_fill(int k, u64 val, int32_t valI, const PathConst &pc, u64 rootv, int32_t &rootI) {
        const u32 s1 = (u32)k; const int B = bitlen(s1);
        bool a1[W], a2[W];
        for (int l = 0; l < W; ++l) { int m = B - (int)pc.bl[l]; u32 t = m >= 0 ? (s1 >> m) : 0u; a1[l] = t == pc.c2[l]; a2[l] = t == pc.c2[l] + 1u; }
        const u64 OL = ballot(a1), OR = ballot(a2);
        const u32 sl = (s1 - 2u) >> 1;
        const u64 selfL = (s1 & 1u) ? 0ull : (1ull << sl), selfR = (s1 & 1u) ? (1ull << sl) : 0ull;
        for (int l = 0; l < W; ++l) { a1[l] = val > L[l]; a2[l] = val > R[l]; }
        const int h = __builtin_popcountll(ballot(a1) & OL & ~selfL) + __builtin_popcountll(ballot(a2) & OR & ~selfR) + (sgt64(val, rootv) ? 1 : 0);
        if (h > 0) {
            u64 f[W]; int32_t fI[W];
            for (int l = 0; l < W; ++l) { bool odd = l & 1; f[l] = odd ? L[pc.addrF[l]] : R[pc.addrF[l]]; fI[l] = odd ? IL[pc.addrF[l]] : IR[pc.addrF[l]]; }
            const u64 mlt = ~0ull << ((1u << (B - h - 1)) - 1u);
            for (int l = 0; l < W; ++l) {
                if (((OL & mlt) >> l) & 1) { L[l] = f[l]; IL[l] = fI[l]; }
                if (((OR & mlt) >> l) & 1) { R[l] = f[l]; IR[l] = fI[l]; }
            }
            if (h == B - 1) {
                if (OL & 1ull) { L[0] = rootv; IL[0] = rootI; }
                if (OR & 1ull) { R[0] = rootv; IR[0] = rootI; }
                rootI = valI;
                R[63] = val; IR[63] = valI;
                return val;
            }
        }
        const u32 x = (s1 >> h) - 1u; const int xl = (int)((x - 1u) >> 1);
        if (x & 1u) { L[xl] = val; IL[xl] = valI; } else { R[xl] = val; IR[xl] = valI; }
        return rootv;
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


