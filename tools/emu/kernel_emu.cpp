// Host model of the lean search kernel's level-0 loop (hnsw_pq_fast_kernel, LOGRES, ef = efSearch = k = 128) for
// one query, lane by lane, on the wave heap of tools/emu/wave_emu.h: the heap as the visited set, the fill / full
// push loops, the log of tied evictions and the final selection from the heap's entries plus that log. Test
// infrastructure (tests/test_kernel_model.py): g++ -O2 -std=c++17 -shared -fPIC kernel_emu.cpp
#include <algorithm>
#include <cstring>

#include "wave_emu.h"

// ---- the lean kernel's level-0 loop (hnsw_pq_fast_kernel, LOGRES, ef = efSearch = k = 128), one query, lane by lane
static u32 ord32(float f) { u32 u; std::memcpy(&u, &f, 4); return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }
static u32 pop_hash(int32_t v) { return (((u32)v & 0xFFFFFFu) * 0x9E3779u) >> 21; }

extern "C" int emu_search_one(const int32_t *nbr0, const uint8_t *codes, int64_t ntotal, int deg0, const float *lut,
                              int32_t nearest, float dnear, int32_t *out_ids, uint32_t *out_keys, int32_t *stats)
{
    static PathConst pc;
    const int ef = 128, k = 128, ef_search = 128, log_cap = 512;
    auto adc = [&](int32_t v) { float r = 0.0f; for (int m = 0; m < 8; ++m) r = r + lut[m * 256 + codes[(size_t)v * 8 + m]]; return ord32(r); };
    Heap hp;
    for (int l = 0; l < W; ++l) { hp.L[l] = kUnused; hp.R[l] = kUnused; hp.IL[l] = -1; hp.IR[l] = -1; }
    const u32 dn = ord32(dnear);
    hp.R[63] = pack(dn, nearest); hp.IR[63] = nearest;
    int kc = 1, nvalid = 1;
    u64 root = pack(dn, nearest); int32_t rootI = nearest;
    std::vector<u64> lg;        // tied evictions (the kernel's log before the heap's entries join it)
    std::vector<int32_t> pushed{nearest}; // every accepted push, for the duplicate check
    int nstep = 0, maxlog = 0;
    int32_t pred = -1;
    u32 popped_bits[W] = {};
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
        auto below_root = [&]() { bool c[W]; for (int l = 0; l < W; ++l) c[l] = dall[l] < hi32(root); return ballot(c); };
        if (kc < ef) { // the heap fills
            while (rem) {
                const int l = __builtin_ctzll(rem); rem &= rem - 1;
                const u32 key = dall[l]; const int32_t idl = v1[l];
                if (hp.holds(idl)) continue;
                ++kc;
                hp.push_fill(kc, pack(key, idl), idl, pc);
                ++nvalid;
                pushed.push_back(idl);
                if (kc == ef) { // the root is read once the heap is full (push_fill does not track it)
                    root = hp.R[63]; rootI = hp.IR[63];
                    break;
                }
            }
        }
        rem &= below_root();
        while (rem) { // the full heap: pop the max, push val; log an evicted entry tied with the new root
            const int l = __builtin_ctzll(rem); rem &= rem - 1;
            const u32 key = dall[l];
            if (key >= hi32(root)) { std::printf("candidate at or above the root at hop %d\n", nstep); return -5; }
            const int32_t idl = v1[l];
            if (hp.holds(idl)) continue;
            const u32 evk = hi32(root); const int32_t evi = rootI;
            nvalid += lo32(root) == kPopLo ? 1 : 0;
            root = hp.replace128(pack(key, idl), idl, pc, rootI);
            rem &= below_root(); // the root fell: links at or above it leave the mask
            if (evk == hi32(root)) lg.push_back(pack(evk, evi));
            pushed.push_back(idl);
        }
        if (kc == ef && (hp.R[63] != root || hp.IR[63] != rootI)) { std::printf("root not current at hop %d\n", nstep); return -4; }
        maxlog = std::max<int>(maxlog, (int)lg.size());
        nstep++;
    }
    // the k results: the heap's entries (node ids) plus the log, every entry below T = the root's key, then the
    // smallest ids at T (log_id_threshold / log_select)
    for (int l = 0; l < W; ++l) {
        if (hp.IL[l] >= 0) lg.push_back(pack(hi32(hp.L[l]), hp.IL[l]));
        if (hp.IR[l] >= 0) lg.push_back(pack(hi32(hp.R[l]), hp.IR[l]));
    }
    const u32 T = kc == ef ? hi32(root) : 0xFFFFFFFFu;
    std::vector<u64> sel, eq;
    for (u64 e : lg) if (hi32(e) == T) eq.push_back(e);
    std::sort(eq.begin(), eq.end());
    for (u64 e : lg) if (hi32(e) < T) sel.push_back(e);
    for (int i = 0; i < (int)eq.size() && (int)sel.size() < k; ++i) sel.push_back(eq[i]);
    std::sort(sel.begin(), sel.end());
    for (int j = 0; j < k; ++j) {
        out_ids[j] = j < (int)sel.size() ? (int32_t)(lo32(sel[j]) ^ 0x80000000u) : -1;
        out_keys[j] = j < (int)sel.size() ? hi32(sel[j]) : 0xFFFFFFFFu;
    }
    // a node pushed twice would be a visited-set failure
    std::sort(pushed.begin(), pushed.end());
    int dups = 0; for (size_t i = 1; i < pushed.size(); ++i) dups += pushed[i] == pushed[i - 1];
    stats[0] = nstep; stats[1] = (int)lg.size(); stats[2] = dups; stats[3] = maxlog + k > log_cap;
    return 0;
}
