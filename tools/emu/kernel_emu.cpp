#include <algorithm>
#include <cstring>
// Host emulation of the lean search kernel's wave-parallel MinimaxHeap (hnsw_pq_fast.hip: Heap::replace128,
// Heap::push_fill, pop_min's slot marking, Heap::holds) against a literal faiss MinimaxHeap that also keeps the
// node id of every slot. Each VGPR is an array of 64 lanes; ballot / readlane / ds_bpermute / inverse_ballot are
// loops. Random push / pop_min sequences with many equal distances; any divergence of keys, ids or the root is
// reported with the step. Diagnostic tool (not product code): g++ -O2 -std=c++17 heap_emu.cpp -o heap_emu
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
        u64 rootv = val; int32_t rI = valI; u32 last = 64u;
        if (Wm) {
            last = 63u - (u32)__builtin_clzll(Wm);
            for (int l = 0; l < W; ++l) {
                const bool atlast = l == (int)last;
                const u64 up = atlast ? val : up0[l]; const int32_t upI = atlast ? valI : up0I[l];
                if ((Wm & lm) >> l & 1) { L[l] = up; IL[l] = upI; }
                if ((Wm & ~lm) >> l & 1) { R[l] = up; IR[l] = upI; }
            }
            if (Wm & 1ull) { rootv = chv[0]; rI = chI[0]; }
        }
        constexpr u64 kHold = (1ull << 63) | (1ull << 31) | (1ull << 15) | (1ull << 7) | (1ull << 3) | (1ull << 1) | 1ull;
        constexpr u64 kAncL = kHold & ~(1ull << 63);
        for (int l = 0; l < W; ++l) t[l] = vnew > L[l];
        const int h = __builtin_popcountll(ballot(t) & kAncL) + (sgt64(vnew, rootv) ? 1 : 0);
        if (h == 0) { L[63] = vnew; IL[63] = vnewI; rootI = rI; return rootv; }
        u64 fl[W]; int32_t flI[W];
        for (int l = 0; l < W; ++l) {
            const u32 k = (u32)l >> 1; const bool moved = ((Wm & lm) >> k) & 1ull; const bool klast = k == last;
            fl[l] = moved ? (klast ? val : chv[l]) : fpre[l]; flI[l] = moved ? (klast ? valI : chI[l]) : fpreI[l];
        }
        const u64 wm = kHold & (~0ull << ((1u << (7 - h)) - 1u));
        for (int l = 0; l < W; ++l) if ((wm >> l) & 1) { L[l] = fl[l]; IL[l] = flI[l]; }
        if (h == 7) { L[0] = rootv; IL[0] = rI; rootI = vnewI; return vnew; }
        const int sx = (1u << (6 - h)) - 1u;
        L[sx] = vnew; IL[sx] = vnewI;
        rootI = rI;
        return rootv;
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
                return val;
            }
        }
        const u32 x = (s1 >> h) - 1u; const int xl = (int)((x - 1u) >> 1);
        if (x & 1u) { L[xl] = val; IL[xl] = valI; } else { R[xl] = val; IR[xl] = valI; }
        return rootv;
    }
};


// ---- the lean kernel's level-0 loop (hnsw_pq_fast_kernel, LOGRES, ef = efSearch = k = 128), one query, lane by lane
static u32 ord32(float f) { u32 u; std::memcpy(&u, &f, 4); return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }
static u32 pop_hash(int32_t v) { return ((u32)v * 2654435761u) >> 21; }

extern "C" int emu_search_one(const int32_t *nbr0, const uint8_t *codes, int64_t ntotal, int deg0, const float *lut,
                              int32_t nearest, float dnear, int32_t *out_ids, uint32_t *out_keys, int32_t *stats)
{
    static PathConst pc;
    const int ef = 128, k = 128, ef_search = 128, log_cap = 2048;
    auto adc = [&](int32_t v) { float r = 0.0f; for (int m = 0; m < 8; ++m) r = r + lut[m * 256 + codes[(size_t)v * 8 + m]]; return ord32(r); };
    Heap hp;
    for (int l = 0; l < W; ++l) { hp.L[l] = kUnused; hp.R[l] = kUnused; hp.IL[l] = -1; hp.IR[l] = -1; }
    const u32 dn = ord32(dnear);
    hp.R[63] = pack(dn, nearest); hp.IR[63] = nearest;
    int kc = 1, nvalid = 1;
    u64 root = pack(dn, nearest); int32_t rootI = nearest;
    std::vector<u64> lg; lg.push_back(root);
    int nstep = 0, maxlog = 1;
    int32_t pred = -1;
    u32 popped_bits[W] = {};
    int32_t prow = -1; // node whose row praw holds
    while (nvalid > 0) {
        if (nstep > ntotal) return -1;
        // pop_min
        bool vL[W], vR[W]; u32 cL[W], cR[W], pk[W]; bool pickR[W];
        u32 d0 = 0xFFFFFFFFu;
        for (int l = 0; l < W; ++l) {
            vL[l] = lo32(hp.L[l]) != kPopLo; vR[l] = lo32(hp.R[l]) != kPopLo;
            cL[l] = vL[l] ? hi32(hp.L[l]) : 0xFFFFFFFFu; cR[l] = vR[l] ? hi32(hp.R[l]) : 0xFFFFFFFFu;
            pickR[l] = cR[l] < cL[l] || (cR[l] == cL[l] && l != 63);
            pk[l] = pickR[l] ? cR[l] : cL[l]; d0 = std::min(d0, pk[l]);
        }
        const u64 rightm = ballot(pickR);
        bool t[W]; for (int l = 0; l < W; ++l) t[l] = pk[l] == d0;
        const u64 tiedm = ballot(t) & ~(rightm & (1ull << 63));
        int wl = 63; bool wR = true;
        if (tiedm) { wl = 63 - __builtin_clzll(tiedm); wR = (rightm >> wl) & 1ull; }
        const int32_t v0 = (int32_t)(lo32(wR ? hp.R[wl] : hp.L[wl]) ^ 0x80000000u);
        if (v0 < 0 || v0 >= ntotal) { std::printf("bad v0 %d at hop %d (d0 %08x nvalid %d)\n", v0, nstep, d0, nvalid); return -2; }
        if (wR) hp.R[wl] = (hp.R[wl] & ~0xFFFFFFFFull) | kPopLo; else hp.L[wl] = (hp.L[wl] & ~0xFFFFFFFFull) | kPopLo;
        if (wl == 63 && wR) root = (root & ~0xFFFFFFFFull) | kPopLo;
        nvalid--;
        int below = 0; for (int l = 0; l < W; ++l) below += (hi32(hp.L[l]) < d0) + (hi32(hp.R[l]) < d0);
        if (below >= ef_search) break;
        { const u32 h0 = pop_hash(v0); popped_bits[(h0 >> 5) & 63u] |= 1u << (h0 & 31u); }
        int32_t v1[W]; u32 dall[W];
        for (int l = 0; l < W; ++l) { v1[l] = l < deg0 ? nbr0[(size_t)v0 * deg0 + l] : -1; }
        int jmax = 64; for (int l = 0; l < W; ++l) if (v1[l] < 0) { jmax = l; break; }
        for (int l = 0; l < W; ++l) dall[l] = (l < jmax) ? adc(v1[l]) : 0u;
        // prediction (only its validity matters here)
        {
            u32 mm = 0xFFFFFFFFu; int32_t pr = -1;
            for (int l = 0; l < W; ++l) {
                const u32 hv = pop_hash(v1[l]);
                const bool kp = (popped_bits[(hv >> 5) & 63u] >> (hv & 31u)) & 1u;
                const u32 dp = (l < jmax && !kp) ? dall[l] : 0xFFFFFFFFu;
                const u32 hL = lo32(hp.L[l]) != kPopLo ? hi32(hp.L[l]) : 0xFFFFFFFFu;
                const u32 hR = lo32(hp.R[l]) != kPopLo ? hi32(hp.R[l]) : 0xFFFFFFFFu;
                u32 mk = std::min(dp, std::min(hL, hR));
                const int32_t mid = dp == mk ? v1[l] : (hL == mk ? (int32_t)(lo32(hp.L[l]) ^ 0x80000000u) : (int32_t)(lo32(hp.R[l]) ^ 0x80000000u));
                if (mk < mm) { mm = mk; pr = mid; }
            }
            pred = mm != 0xFFFFFFFFu ? pr : -1;
            if (pred >= ntotal || (mm != 0xFFFFFFFFu && pred < 0)) { std::printf("bad pred %d at hop %d\n", pred, nstep); return -3; }
        }
        u64 rem = jmax >= 64 ? ~0ull : ((1ull << jmax) - 1ull);
        if (kc == ef) { bool c[W]; for (int l = 0; l < W; ++l) c[l] = dall[l] < hi32(root); rem &= ballot(c); }
        int sn = 0;
        while (rem) {
            const int l = __builtin_ctzll(rem); rem &= rem - 1;
            const u32 key = dall[l];
            if (kc == ef && key >= hi32(root)) continue;
            const int32_t idl = v1[l];
            if (hp.holds(idl)) continue;
            const u64 val = pack(key, idl);
            if (kc == ef) {
                if (lo32(root) != kPopLo) --nvalid;
                root = hp.replace128(val, idl, pc, rootI);
                hp.IR[63] = rootI;
            } else {
                ++kc;
                root = hp.push_fill(kc, val, idl, pc, root, rootI);
                hp.IR[63] = rootI;
            }
            ++nvalid;
            lg.push_back(val); ++sn;
        }
        hp.R[63] = root;
        maxlog = std::max<int>(maxlog, (int)lg.size());
        nstep++;
    }
    // the k results: sort the log, keep k smallest with T = root key (emulating log_select's tie rule)
    const u32 T = kc == ef ? hi32(root) : 0xFFFFFFFFu;
    std::vector<u64> sel;
    int nlt = 0; for (u64 e : lg) nlt += hi32(e) < T;
    std::vector<u64> eq; for (u64 e : lg) if (hi32(e) == T) eq.push_back(e);
    std::sort(eq.begin(), eq.end());
    for (u64 e : lg) if (hi32(e) < T) sel.push_back(e);
    for (int i = 0; i < (int)eq.size() && (int)sel.size() < k; ++i) sel.push_back(eq[i]);
    std::sort(sel.begin(), sel.end());
    for (int j = 0; j < k; ++j) {
        out_ids[j] = j < (int)sel.size() ? (int32_t)(lo32(sel[j]) ^ 0x80000000u) : -1;
        out_keys[j] = j < (int)sel.size() ? hi32(sel[j]) : 0xFFFFFFFFu;
    }
    // duplicates in the log would be a visited-set failure
    std::vector<int32_t> ids; for (u64 e : lg) ids.push_back((int32_t)(lo32(e) ^ 0x80000000u));
    std::sort(ids.begin(), ids.end());
    int dups = 0; for (size_t i = 1; i < ids.size(); ++i) dups += ids[i] == ids[i - 1];
    stats[0] = nstep; stats[1] = (int)lg.size(); stats[2] = dups; stats[3] = maxlog > log_cap;
    return 0;
}
