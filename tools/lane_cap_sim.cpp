// Lock-step model of a capped lane walk (tools/lane_cap_sim.py runs it): rays
// (u32 n, then n x (o.xyz, d.xyz) f32, in GPU trace order) are taken 64 at a
// time; every lane walks the single-leaf TLAS's instances in order and each
// BLAS in the reference's DFS (one node per step).  For a cap K on a lane's
// steps, a lane that reaches K leaves the walk (its ray would be finished by a
// one-ray-per-wave pass); the wave's steps at an instance are its slowest
// remaining lane's.  Prints, per K: wave steps per 64 rays, capped rays per
// 64 rays, and the capped rays' full DFS steps (their wave-walk work).
// A probe only: links the oracle's restatement as its traversal model.
#include "../oracle/cpu_ref.cpp"
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
    /* one ray's walk over the instances in TLAS order from depth `depth`, one
     * node per step, stopping after `cap` steps: per-instance steps into st
     * (if given); returns the steps taken, depth holds the depth reached */
    auto walk = [&](uint32_t i, float& depth, uint32_t cap, uint32_t* st) -> uint32_t {
        V3 o = mk(od[6*i], od[6*i+1], od[6*i+2]), d = mk(od[6*i+3], od[6*i+4], od[6*i+5]);
        uint32_t total = 0;
        for (uint32_t k = 0; k < nI && total < cap; ++k) {
            const Instance& in = S.inst[T.idx[root.lf + k]];
            if (slab(in.bounds, o, d, depth) == kFarAway) continue;
            V4 tp = mul(in.Minv, v4(o, 1.0f)), td = mul(in.Minv, v4(d, 0.0f));
            V3 oo = xyz(tp) / tp.w, dd = xyz(td);
            const Bvh& b = in.blas->bvh;
            const Node& r = b.nodes[0];
            const auto& tris = in.blas->mesh->tris;
            if (r.cnt) { for (uint32_t q = 0; q < r.cnt; ++q) { float u, v; hitTri(tris[b.idx[r.lf + q]], oo, dd, depth, u, v); } continue; }
            uint32_t cn = r.lf, cf = r.lf + 1;
            float dn = slab(b.nodes[cn].box, oo, dd, depth), df = slab(b.nodes[cf].box, oo, dd, depth);
            if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
            if (dn == kFarAway) continue;
            std::vector<uint32_t> stk; if (df != kFarAway) stk.push_back(cf);
            uint32_t node = cn, s = 0;
            for (;;) {
                if (total + s >= cap) break;
                ++s;
                const Node& nd = b.nodes[node];
                bool pop = false;
                if (nd.cnt) {
                    for (uint32_t q = 0; q < nd.cnt; ++q) { float u, v; hitTri(tris[b.idx[nd.lf + q]], oo, dd, depth, u, v); }
                    pop = true;
                } else {
                    uint32_t a = nd.lf, c = nd.lf + 1;
                    float e0 = slab(b.nodes[a].box, oo, dd, depth), e1 = slab(b.nodes[c].box, oo, dd, depth);
                    if (e0 > e1) { std::swap(e0, e1); std::swap(a, c); }
                    if (e0 == kFarAway) pop = true; else { node = a; if (e1 != kFarAway) stk.push_back(c); }
                }
                if (pop) { if (stk.empty()) break; node = stk.back(); stk.pop_back(); }
            }
            if (st) st[k] = s;
            total += s;
        }
        return total;
    };
    /* per ray, per instance (TLAS order): DFS steps with the depth the earlier instances left */
    std::vector<uint32_t> steps((size_t)n * nI, 0);
    #pragma omp parallel for schedule(dynamic, 64)
    for (long long i = 0; i < (long long)n; ++i) {
        float depth = kFarAway;
        walk((uint32_t)i, depth, 0xffffffffu, &steps[(size_t)i * nI]);
    }
    const uint32_t G = n / 64;
    std::vector<uint32_t> caps = {1u << 30, 512, 384, 256, 192, 160, 128, 96, 64, 48, 32};
    for (uint32_t K : caps) {
        double wsteps = 0, capped = 0, cappedWork = 0, laneSteps = 0, restart = 0;
        if (K < (1u << 30)) {
            #pragma omp parallel for schedule(dynamic, 64) reduction(+ : restart)
            for (long long i = 0; i < (long long)(G * 64); ++i) {
                uint32_t tot = 0;
                for (uint32_t k = 0; k < nI; ++k) tot += steps[(size_t)i * nI + k];
                if (tot <= K) continue;
                float depth = kFarAway;
                walk((uint32_t)i, depth, K, nullptr);
                restart += walk((uint32_t)i, depth, 0xffffffffu, nullptr);
            }
        }
        std::vector<uint32_t> rem;          /* capped rays' steps left, in ray order */
        for (uint32_t g = 0; g < G; ++g) {
            uint32_t cum[64] = {0};
            bool cap[64] = {false};
            for (uint32_t k = 0; k < nI; ++k) {
                uint32_t mx = 0;
                for (int l = 0; l < 64; ++l) {
                    if (cap[l]) continue;
                    const uint32_t s = steps[(size_t)(g * 64 + l) * nI + k];
                    if (!s) continue;
                    const uint32_t room = K - cum[l];
                    const uint32_t t = s < room ? s : room;
                    mx = t > mx ? t : mx;
                    laneSteps += t;
                    if (s >= room && cum[l] + s > K) { cap[l] = true; cum[l] = K; } else cum[l] += s;
                }
                wsteps += mx;
            }
            for (int l = 0; l < 64; ++l) if (cap[l]) {
                capped += 1;
                uint32_t tot = 0;
                for (uint32_t k = 0; k < nI; ++k) tot += steps[(size_t)(g * 64 + l) * nI + k];
                cappedWork += tot;
                rem.push_back(tot - K);
            }
        }
        /* a lane-walk continuation pass over the capped rays, 64 per wave in
         * ray order (compacted): its wave steps are each group's longest rest */
        double cont = 0;
        for (size_t q = 0; q < rem.size(); q += 64) {
            uint32_t mx = 0;
            for (size_t l = q; l < rem.size() && l < q + 64; ++l) mx = rem[l] > mx ? rem[l] : mx;
            cont += mx;
        }
        printf("cap %10u: lane continuation wave steps/64 rays %.2f (total %.2f)\n", K, cont / G, wsteps / G + cont / G);
        printf("cap %10u: wave steps/64 rays %.2f  lane util %.3f  capped rays/64 %.4f (%.4f%%)  their DFS steps/64 %.2f  restart steps/64 %.2f  left after cap/64 %.2f\n", K,
               wsteps / G, laneSteps / (wsteps * 64.0), capped / G, 100.0 * capped / (G * 64.0), cappedWork / G, restart / G,
               (cappedWork - capped * K) / G);
    }
    return 0;
}
