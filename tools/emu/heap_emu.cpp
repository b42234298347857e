// Host emulation of the lean search kernel's wave-parallel MinimaxHeap (tools/emu/wave_emu.h: Heap::replace128,
// Heap::push_fill, pop_min's slot marking, Heap::holds) against a literal faiss MinimaxHeap that also keeps the node
// id of every slot: random push / pop_min sequences with many equal distances; any divergence of keys, ids, the root
// or heap membership is reported with the step. Test infrastructure: g++ -O2 -std=c++17 heap_emu.cpp -o heap_emu
#include "wave_emu.h"

// literal faiss MinimaxHeap (0-based arrays, 1-based algorithms) with ids of popped slots kept aside
struct Ref {
    int n = 128, k = 0, nvalid = 0;
    explicit Ref(int n_ = 128) : n(n_) {}
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
        // every other trial: a smaller heap (ef < 128), the kernel's general Heap::pop / Heap::push path
        const int n = (t & 1) ? 2 + (int)(rng() % 126) : 128;
        Heap hp; Ref ref(n);
        for (int l = 0; l < W; ++l) { hp.L[l] = kUnused; hp.R[l] = kUnused; hp.IL[l] = -1; hp.IR[l] = -1; }
        const int nd = 2 + (int)(rng() % 40); // few distinct distances: ties
        int32_t next_id = 0;
        u64 root = 0; int32_t rootI = -1; int kc = 0;
        auto push = [&](u32 key, int32_t id) {
            // the kernel: full heap -> reject at or above the root, else replace; filling -> push_fill
            const bool ok_ref = ref.push(id, key);
            if (kc == 0) { // first push: the entry (hp.R[63] = root)
                hp.R[63] = pack(key, id); hp.IR[63] = id; root = hp.R[63]; rootI = id; kc = 1;
            } else if (kc == n) {
                if (key >= hi32(root)) { if (ok_ref) { std::printf("trial %d: reject mismatch\n", t); std::exit(1); } return; }
                if (n == 128) {
                    root = hp.replace128(pack(key, id), id, pc, rootI);
                } else {
                    hp.pop(kc); hp.push(kc, pack(key, id), id); root = hp.R[63]; rootI = hp.IR[63];
                }
            } else if (n == 128) {
                ++kc; hp.push_fill(kc, pack(key, id), id, pc); root = hp.R[63]; rootI = hp.IR[63];
            } else {
                ++kc; hp.push(kc, pack(key, id), id); root = hp.R[63]; rootI = hp.IR[63];
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
