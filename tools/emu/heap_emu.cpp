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

// literal faiss MinimaxHeap (0-based arrays, 1-based algorithms) with ids of popped slots kept aside
struct Ref {
    int n = 128, k = 0, nvalid = 0;
    std::vector<u32> dis = std::vector<u32>(128); std::vector<int32_t> ids = std::vector<int32_t>(128), node = std::vector<int32_t>(128);
    static bool cmp2(u32 a1, u32 b1, int32_t a2, int32_t b2) { return a1 > b1 || (a1 == b1 && a2 > b2); }
    void heap_pop(int kk) {
        u32 *bv = dis.data() - 1; int32_t *bi = ids.data() - 1, *bn = node.data() - 1;
        u32 v = bv[kk]; int32_t id = bi[kk];
        int i = 1;
        for (;;) {
            int i1 = i << 1, i2 = i1 + 1;
            if (i1 > kk) break;
            if (i2 == kk + 1 || cmp2(bv[i1], bv[i2], bi[i1], bi[i2])) {
                if (cmp2(v, bv[i1], id, bi[i1])) break;
                bv[i] = bv[i1]; bi[i] = bi[i1]; bn[i] = bn[i1]; i = i1;
            } else {
                if (cmp2(v, bv[i2], id, bi[i2])) break;
                bv[i] = bv[i2]; bi[i] = bi[i2]; bn[i] = bn[i2]; i = i2;
            }
        }
        bv[i] = bv[kk]; bi[i] = bi[kk]; bn[i] = bn[kk];
    }
    void heap_push(int kk, u32 v, int32_t id) {
        u32 *bv = dis.data() - 1; int32_t *bi = ids.data() - 1, *bn = node.data() - 1;
        int i = kk;
        while (i > 1) { int f = i >> 1; if (!cmp2(v, bv[f], id, bi[f])) break; bv[i] = bv[f]; bi[i] = bi[f]; bn[i] = bn[f]; i = f; }
        bv[i] = v; bi[i] = id; bn[i] = id;
    }
    bool push(int32_t i, u32 v) {
        if (k == n) { if (v >= dis[0]) return false; if (ids[0] != -1) --nvalid; heap_pop(k--); }
        heap_push(++k, v, i); ++nvalid; return true;
    }
    int pop_min() {
        int i = k - 1; while (i >= 0 && ids[i] == -1) --i;
        if (i < 0) return -1;
        int imin = i; u32 vmin = dis[i];
        for (--i; i >= 0; --i) if (ids[i] != -1 && dis[i] < vmin) { vmin = dis[i]; imin = i; }
        int r = ids[imin]; ids[imin] = -1; --nvalid; return imin;
    }
};

static u64 slot_key(const Heap &h, int s) { if (s == 0) return h.R[63]; int o = (s - 1) >> 1; return (s & 1) ? h.L[o] : h.R[o]; }
static int32_t slot_id(const Heap &h, int s) { if (s == 0) return h.IR[63]; int o = (s - 1) >> 1; return (s & 1) ? h.IL[o] : h.IR[o]; }
static u64 &slot_key_ref(Heap &h, int s) { if (s == 0) return h.R[63]; int o = (s - 1) >> 1; return (s & 1) ? h.L[o] : h.R[o]; }

int main(int argc, char **argv)
{
    const int trials = argc > 1 ? std::atoi(argv[1]) : 2000;
    PathConst pc;
    std::mt19937_64 rng(7);
    long checks = 0;
    for (int t = 0; t < trials; ++t) {
        Heap hp; Ref ref;
        for (int l = 0; l < W; ++l) { hp.L[l] = kUnused; hp.R[l] = kUnused; hp.IL[l] = -1; hp.IR[l] = -1; }
        const int nd = 2 + (int)(rng() % 40); // few distinct distances: ties
        int32_t next_id = 0;
        u64 root = 0; int32_t rootI = -1; int kc = 0;
        auto push = [&](u32 key, int32_t id) {
            // the kernel: full heap -> reject at or above the root, else replace; filling -> push_fill
            const bool ok_ref = ref.push(id, key);
            if (kc == 0) { // first push: the entry (hp.R[63] = root)
                hp.R[63] = pack(key, id); hp.IR[63] = id; root = hp.R[63]; rootI = id; kc = 1;
            } else if (kc == 128) {
                if (key >= hi32(root)) { if (ok_ref) { std::printf("trial %d: reject mismatch\n", t); std::exit(1); } return; }
                root = hp.replace128(pack(key, id), id, pc, rootI); hp.R[63] = root; hp.IR[63] = rootI;
            } else {
                ++kc; root = hp.push_fill(kc, pack(key, id), id, pc, root, rootI); hp.R[63] = root; hp.IR[63] = rootI;
            }
            if (!ok_ref) { std::printf("trial %d: accept mismatch\n", t); std::exit(1); }
        };
        for (int step = 0; step < 2000; ++step) {
            if (rng() % 3 || kc == 0) {
                push((u32)(rng() % nd) + 0x80000000u, next_id++);
            } else { // pop_min as the kernel marks it: the slot's key low word -> kPopLo
                const int s = ref.pop_min();
                if (s < 0) continue;
                u64 &kk = slot_key_ref(hp, s);
                kk = (kk & ~0xFFFFFFFFull) | kPopLo;
                if (s == 0) root = (root & ~0xFFFFFFFFull) | kPopLo;
            }
            for (int s = 0; s < ref.k; ++s) {
                const u64 want = ((u64)ref.dis[s] << 32) | (u32)((u32)ref.ids[s] ^ 0x80000000u);
                if (slot_key(hp, s) != want || slot_id(hp, s) != ref.node[s]) {
                    std::printf("trial %d step %d slot %d: key %016llx want %016llx id %d want %d\n", t, step, s,
                                (unsigned long long)slot_key(hp, s), (unsigned long long)want, slot_id(hp, s), ref.node[s]);
                    std::exit(1);
                }
                ++checks;
            }
            // membership == ids present in the reference heap
            for (int q = 0; q < 4; ++q) {
                const int32_t v = (int32_t)(rng() % (next_id + 1));
                bool in_ref = false;
                for (int s = 0; s < ref.k; ++s) in_ref |= ref.node[s] == v;
                if (hp.holds(v) != in_ref) { std::printf("trial %d step %d: holds(%d) = %d, want %d\n", t, step, v, hp.holds(v), in_ref); std::exit(1); }
            }
        }
    }
    std::printf("ok: %d trials, %ld slot checks\n", trials, checks);
    return 0;
}
