// Closest-hit BLAS node visits per ray with the instances of the single-leaf
// TLAS taken in TLAS order (the reference's) against nearest-world-box-first
// (tools/inst_order_sim.py runs it).  Nearest-first stays exact with a tie
// rule: an instance earlier in TLAS order than the current best hit's accepts
// t <= best (its depth is nextafter(best)), a later one t < best.
// Rays: u32 n, then n x (o.xyz, d.xyz) f32.  Prints visits per ray for both
// orders and checks that the hits agree.
// A probe only: links the oracle's restatement as its traversal model.
#include "../oracle/cpu_ref.cpp"
#include <algorithm>
#include <cmath>
static uint32_t bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
int main(int argc, char** argv) {
    orc_scene* h = orc_scene_create(getenv("SURF_ASSETS") ? getenv("SURF_ASSETS") : "assets", getenv("SCENE_VARIANT") ? atoi(getenv("SCENE_VARIANT")) : 0);
    Scene& S = *h->s;
    FILE* f = fopen(argv[1], "rb"); uint32_t n = 0;
    if (!f || fread(&n, 4, 1, f) != 1) return 1;
    std::vector<float> od(6 * (size_t)n);
    if (fread(od.data(), 4, od.size(), f) != od.size()) return 1;
    fclose(f);
    const Bvh& T = S.tlas;
    const Node& root = T.nodes[0];
    const uint32_t nI = root.cnt;
    /* one instance's closest-hit walk at depth `depth` (accepting t < depth): visits, hit */
    auto inst = [&](uint32_t k, V3 o, V3 d, float& depth, float& hu, float& hv, uint32_t& prim, double& visits) -> bool {
        const Instance& in = S.inst[T.idx[root.lf + k]];
        if (slab(in.bounds, o, d, depth) == kFarAway) return false;
        V4 tp = mul(in.Minv, v4(o, 1.0f)), td = mul(in.Minv, v4(d, 0.0f));
        V3 oo = xyz(tp) / tp.w, dd = xyz(td);
        const Bvh& b = in.blas->bvh;
        const Node& r = b.nodes[0];
        const auto& tris = in.blas->mesh->tris;
        bool hit = false;
        auto leaf = [&](const Node& nd) {
            for (uint32_t q = 0; q < nd.cnt; ++q) {
                float u, v;
                if (hitTri(tris[b.idx[nd.lf + q]], oo, dd, depth, u, v)) { hit = true; hu = u; hv = v; prim = b.idx[nd.lf + q]; }
            }
        };
        if (r.cnt) { leaf(r); return hit; }
        uint32_t cn = r.lf, cf = r.lf + 1;
        float dn = slab(b.nodes[cn].box, oo, dd, depth), df = slab(b.nodes[cf].box, oo, dd, depth);
        if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
        if (dn == kFarAway) return false;
        std::vector<uint32_t> stk; if (df != kFarAway) stk.push_back(cf);
        uint32_t node = cn;
        for (;;) {
            visits += 1;
            const Node& nd = b.nodes[node];
            bool pop = false;
            if (nd.cnt) { leaf(nd); pop = true; }
            else {
                uint32_t a = nd.lf, c = nd.lf + 1;
                float e0 = slab(b.nodes[a].box, oo, dd, depth), e1 = slab(b.nodes[c].box, oo, dd, depth);
                if (e0 > e1) { std::swap(e0, e1); std::swap(a, c); }
                if (e0 == kFarAway) pop = true; else { node = a; if (e1 != kFarAway) stk.push_back(c); }
            }
            if (pop) { if (stk.empty()) break; node = stk.back(); stk.pop_back(); }
        }
        return hit;
    };
    double va = 0, vb = 0;
    uint64_t mismatch = 0;
    #pragma omp parallel for schedule(dynamic, 256) reduction(+ : va, vb, mismatch)
    for (long long i = 0; i < (long long)n; ++i) {
        V3 o = mk(od[6*i], od[6*i+1], od[6*i+2]), d = mk(od[6*i+3], od[6*i+4], od[6*i+5]);
        /* (a) TLAS order */
        float da = kFarAway, ua = 0, wa = 0; uint32_t pa = ~0u, ka = ~0u;
        for (uint32_t k = 0; k < nI; ++k) if (inst(k, o, d, da, ua, wa, pa, va)) ka = k;
        /* (b) nearest world box first, tie rule by TLAS place */
        std::vector<std::pair<float, uint32_t>> ord;
        for (uint32_t k = 0; k < nI; ++k) {
            const float e = slab(S.inst[T.idx[root.lf + k]].bounds, o, d, kFarAway);
            if (e != kFarAway) ord.push_back({e, k});
        }
        std::stable_sort(ord.begin(), ord.end());
        float db = kFarAway, ub = 0, wb = 0; uint32_t pb = ~0u, kb = ~0u;
        for (auto& [e, k] : ord) {
            float dk = (kb != ~0u && k < kb) ? std::nextafter(db, kFarAway) : db;
            if (e >= dk) continue;
            float u = ub, w = wb; uint32_t p = pb;
            if (inst(k, o, d, dk, u, w, p, vb)) { db = dk; ub = u; wb = w; pb = p; kb = k; }
        }
        if (ka != kb || bits(da) != bits(db) || pa != pb || bits(ua) != bits(ub) || bits(wa) != bits(wb)) ++mismatch;
    }
    printf("rays %u  visits per ray: TLAS order %.2f, nearest box first %.2f (%.1f %%)  hit mismatches %llu\n", n, va / n, vb / n,
           100.0 * (vb - va) / va, (unsigned long long)mismatch);
    return 0;
}
