// scene.cpp -- BVH build (binned SAH, 4 prims per leaf like pbrt's default maxnodeprims,
// accelerators/bvh.cpp:547-550) and TessellateSurfacePoints (see scene.h).
#include "scene.h"

#include "geom.h"
#include "tessellate.h"
#include "texture.h"

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstring>
#include <thread>

namespace mpss {

// ------------------------------------------------------------------------------- BVH
namespace {

struct PrimInfo {
    float lo[3], hi[3], c[3];
    int tri;
};

struct BuildCtx {
    std::vector<PrimInfo> prims;
    std::vector<BvhNode> nodes;
    std::vector<int> order;
};

void bounds_of(const std::vector<PrimInfo> &p, int b, int e, float *lo, float *hi, bool centroid) {
    for (int k = 0; k < 3; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (int i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k) {
            const float a = centroid ? p[i].c[k] : p[i].lo[k], z = centroid ? p[i].c[k] : p[i].hi[k];
            lo[k] = std::min(lo[k], a);
            hi[k] = std::max(hi[k], z);
        }
}

float area_of(const float *lo, const float *hi) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0.f;
    return 2.f * (dx * dy + dy * dz + dz * dx);
}

int build_rec(BuildCtx &c, int b, int e) {
    const int me = (int)c.nodes.size();
    c.nodes.emplace_back();
    float lo[3], hi[3];
    bounds_of(c.prims, b, e, lo, hi, false);
    const int n = e - b;
    auto make_leaf = [&] {
        BvhNode &nd = c.nodes[me];
        memcpy(nd.bmin, lo, sizeof(lo));
        memcpy(nd.bmax, hi, sizeof(hi));
        nd.offset = (int32_t)c.order.size();
        nd.nprims = (uint16_t)n;
        nd.axis = 0;
        for (int i = b; i < e; ++i) c.order.push_back(c.prims[i].tri);
        return me;
    };
    if (n <= 4) return make_leaf();
    float clo[3], chi[3];
    bounds_of(c.prims, b, e, clo, chi, true);
    int axis = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
    if (chi[axis] <= clo[axis]) return make_leaf();
    // 16-bin SAH
    constexpr int NBIN = 16;
    int cnt[NBIN] = {};
    float blo[NBIN][3], bhi[NBIN][3];
    for (int i = 0; i < NBIN; ++i)
        for (int k = 0; k < 3; ++k) {
            blo[i][k] = INFINITY;
            bhi[i][k] = -INFINITY;
        }
    const float scale = NBIN / (chi[axis] - clo[axis]);
    auto bin_of = [&](const PrimInfo &p) {
        return std::min(NBIN - 1, std::max(0, (int)((p.c[axis] - clo[axis]) * scale)));
    };
    for (int i = b; i < e; ++i) {
        const int bi = bin_of(c.prims[i]);
        cnt[bi]++;
        for (int k = 0; k < 3; ++k) {
            blo[bi][k] = std::min(blo[bi][k], c.prims[i].lo[k]);
            bhi[bi][k] = std::max(bhi[bi][k], c.prims[i].hi[k]);
        }
    }
    float best = INFINITY;
    int best_split = -1;
    for (int s = 1; s < NBIN; ++s) {
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int nl = 0, nr = 0;
        for (int i = 0; i < NBIN; ++i) {
            float *L = i < s ? llo : rlo, *H = i < s ? lhi : rhi;
            (i < s ? nl : nr) += cnt[i];
            for (int k = 0; k < 3; ++k) {
                L[k] = std::min(L[k], blo[i][k]);
                H[k] = std::max(H[k], bhi[i][k]);
            }
        }
        if (!nl || !nr) continue;
        const float cost = nl * area_of(llo, lhi) + nr * area_of(rlo, rhi);
        if (cost < best) {
            best = cost;
            best_split = s;
        }
    }
    int mid;
    if (best_split < 0) {
        mid = (b + e) / 2;
        std::nth_element(c.prims.begin() + b, c.prims.begin() + mid, c.prims.begin() + e,
                         [&](const PrimInfo &x, const PrimInfo &y) { return x.c[axis] < y.c[axis]; });
    } else {
        mid = (int)(std::partition(c.prims.begin() + b, c.prims.begin() + e,
                                   [&](const PrimInfo &p) { return bin_of(p) < best_split; }) -
                    c.prims.begin());
        if (mid == b || mid == e) mid = (b + e) / 2;
    }
    build_rec(c, b, mid);
    const int second = build_rec(c, mid, e);
    BvhNode &nd = c.nodes[me];
    memcpy(nd.bmin, lo, sizeof(lo));
    memcpy(nd.bmax, hi, sizeof(hi));
    nd.offset = second;
    nd.nprims = 0;
    nd.axis = (uint16_t)axis;
    return me;
}

}  // namespace

void build_bvh(SceneData &s) {
    BuildCtx c;
    s.tri_mesh.clear();
    s.tri_local.clear();
    for (size_t m = 0; m < s.meshes.size(); ++m) {
        const Mesh &mesh = s.meshes[m];
        const int nt = (int)mesh.idx.size() / 3;
        for (int t = 0; t < nt; ++t) {
            PrimInfo p;
            for (int k = 0; k < 3; ++k) {
                p.lo[k] = INFINITY;
                p.hi[k] = -INFINITY;
            }
            for (int v = 0; v < 3; ++v) {
                const float *q = &mesh.P[3 * (size_t)mesh.idx[3 * t + v]];
                for (int k = 0; k < 3; ++k) {
                    p.lo[k] = std::min(p.lo[k], q[k]);
                    p.hi[k] = std::max(p.hi[k], q[k]);
                }
            }
            for (int k = 0; k < 3; ++k) p.c[k] = .5f * p.lo[k] + .5f * p.hi[k];
            p.tri = (int)s.tri_mesh.size();
            s.tri_mesh.push_back((int32_t)m);
            s.tri_local.push_back(t);
            c.prims.push_back(p);
        }
    }
    if (c.prims.empty()) throw Error(-1, "scene has no triangles");
    c.nodes.reserve(2 * c.prims.size());
    build_rec(c, 0, (int)c.prims.size());
    s.bvh = std::move(c.nodes);
    s.tris.resize(c.order.size());
    for (size_t i = 0; i < c.order.size(); ++i) {
        const int g = c.order[i];
        const Mesh &mesh = s.meshes[s.tri_mesh[g]];
        const int t = s.tri_local[g];
        const float *p1 = &mesh.P[3 * (size_t)mesh.idx[3 * t]];
        const float *p2 = &mesh.P[3 * (size_t)mesh.idx[3 * t + 1]];
        const float *p3 = &mesh.P[3 * (size_t)mesh.idx[3 * t + 2]];
        TriRec &r = s.tris[i];
        for (int k = 0; k < 3; ++k) {
            r.p1[k] = p1[k];
            r.e1[k] = p2[k] - p1[k];
            r.e2[k] = p3[k] - p1[k];
        }
        r.tri = g;
        r.mesh = s.tri_mesh[g];
        r.pad = 0;
    }
}

// ------------------------------------------------------------------------------- tessellation
// (the per-triangle code is tessellate.h, shared with the GPU build)

MeshView mesh_view(const Mesh &m) {
    return MeshView{m.P.data(), m.N.empty() ? nullptr : m.N.data(), m.S.empty() ? nullptr : m.S.data(),
                    m.uv.empty() ? nullptr : m.uv.data(), m.idx.data(), m.o2w, m.w2o,
                    (int)(m.reverse_orientation ^ m.swaps_handedness)};
}

void tessellate_surface_points(const SceneData &s, float min_dist, bool incenter, std::vector<SurfacePoint> &out,
                               int nthreads, const TexView *const *bump) {
    out.clear();
    struct Job {
        int mesh, t0, t1;
        std::vector<SurfacePoint> pts;
    };
    std::vector<Job> jobs;
    for (size_t m = 0; m < s.meshes.size(); ++m) {
        const int nt = (int)s.meshes[m].idx.size() / 3;
        for (int t0 = 0; t0 < nt; t0 += 512) jobs.push_back(Job{(int)m, t0, std::min(nt, t0 + 512), {}});
    }
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<int> next{0};
    auto work = [&] {
        for (int j; (j = next.fetch_add(1)) < (int)jobs.size();) {
            Job &job = jobs[j];
            const Mesh &m = s.meshes[job.mesh];
            const MeshView mv = mesh_view(m);
            for (int t = job.t0; t < job.t1; ++t) {
                const TessTri tr = tess_tri(mv, t, min_dist);
                const TexView *bt = bump ? bump[m.material] : nullptr;
                auto shader = [&](BC a, BC b, BC c) {
                    job.pts.push_back(tess_point(mv, t, tr, a, b, c, incenter, bt, m.material, min_dist));
                };
                tessellator(tr.tfe0, tr.tfe1, tr.tfe2, tr.tfc, shader);
            }
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; ++i) th.emplace_back(work);
    for (auto &x : th) x.join();
    size_t total = 0;
    for (auto &j : jobs) total += j.pts.size();
    out.reserve(total);
    for (auto &j : jobs) out.insert(out.end(), j.pts.begin(), j.pts.end());
}

// ------------------------------------------------------------------------------- camera bins
namespace {
bool invert4(const double *m, double *out) {  // Gauss-Jordan with partial pivoting
    double a[4][8];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c) a[r][c] = c < 4 ? m[4 * r + c] : (c - 4 == r ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int piv = c;
        for (int r = c + 1; r < 4; ++r)
            if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
        if (a[piv][c] == 0.0) return false;
        if (piv != c)
            for (int k = 0; k < 8; ++k) std::swap(a[c][k], a[piv][k]);
        const double inv = 1.0 / a[c][c];
        for (int k = 0; k < 8; ++k) a[c][k] *= inv;
        for (int r = 0; r < 4; ++r)
            if (r != c && a[r][c] != 0.0) {
                const double f = a[r][c];
                for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
            }
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out[4 * r + c] = a[r][c + 4];
    return true;
}
void xform4(const double *m, const double *p, double *o) {  // o = m (p, 1), 4 components
    for (int r = 0; r < 4; ++r) o[r] = m[4 * r] * p[0] + m[4 * r + 1] * p[1] + m[4 * r + 2] * p[2] + m[4 * r + 3];
}
}  // namespace

void build_camera_bins(const SceneData &s, CameraBins &b) {
    const Camera &cam = s.camera;
    b.w = cam.xres + 1;
    b.h = cam.yres + 1;
    b.off.assign((size_t)b.w * b.h + 1, 0u);
    b.tri.clear();
    b.all.clear();
    double c2w[16], r2c[16], w2c[16], c2r[16];
    for (int k = 0; k < 16; ++k) {
        c2w[k] = cam.camera_to_world[k];
        r2c[k] = cam.raster_to_camera[k];
    }
    const bool ok = invert4(c2w, w2c) && invert4(r2c, c2r);
    // per triangle: its pixel box [x0, x1] x [y0, y1] (inclusive), or a list tag
    enum { kNone = 0, kBox = 1, kAll = 2 };
    const size_t n = s.tris.size();
    std::vector<int> box(4 * n), tag(n, kNone);
    std::vector<double> q2(6 * n), parea(n, 0.0);  // projected vertices (raster x, y) and area
    for (size_t i = 0; i < n; ++i) {
        if (!ok) {
            tag[i] = kAll;
            continue;
        }
        const TriRec &t = s.tris[i];
        double v[3][3];
        for (int k = 0; k < 3; ++k) {
            v[0][k] = t.p1[k];
            v[1][k] = (double)t.p1[k] + (double)t.e1[k];
            v[2][k] = (double)t.p1[k] + (double)t.e2[k];
        }
        int behind = 0, near = 0;
        double lo[2] = {1e300, 1e300}, hi[2] = {-1e300, -1e300};
        for (int j = 0; j < 3; ++j) {
            double pc[4], pr[4];
            xform4(w2c, v[j], pc);
            const double dist = std::sqrt(pc[0] * pc[0] + pc[1] * pc[1] + pc[2] * pc[2]);
            const double eps = 1e-3 * dist;  // (camera rays leave the origin with a positive z)
            if (pc[2] < -eps) ++behind;
            if (pc[2] <= eps) {
                ++near;
                continue;
            }
            xform4(c2r, pc, pr);
            if (!(pr[3] != 0.0)) {
                ++near;
                continue;
            }
            for (int k = 0; k < 2; ++k) {
                const double q = pr[k] / pr[3];
                q2[6 * i + 2 * j + k] = q;
                lo[k] = std::min(lo[k], q);
                hi[k] = std::max(hi[k], q);
            }
        }
        if (behind == 3) continue;  // no point of it has a positive camera z: no camera ray reaches it
        if (near > 0) {
            tag[i] = kAll;
            continue;
        }
        const double x0 = std::floor(lo[0] - kCamBinMargin), x1 = std::floor(hi[0] + kCamBinMargin);
        const double y0 = std::floor(lo[1] - kCamBinMargin), y1 = std::floor(hi[1] + kCamBinMargin);
        if (x1 < 0 || y1 < 0 || x0 > b.w - 1 || y0 > b.h - 1) continue;  // off the sample extent
        const int ix0 = (int)std::max(0.0, x0), ix1 = (int)std::min((double)b.w - 1, x1);
        const int iy0 = (int)std::max(0.0, y0), iy1 = (int)std::min((double)b.h - 1, y1);
        if ((int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) > kCamBinMaxArea) {
            tag[i] = kAll;
            continue;
        }
        tag[i] = kBox;
        const double *q = &q2[6 * i];
        parea[i] = 0.5 * ((q[2] - q[0]) * (q[5] - q[1]) - (q[4] - q[0]) * (q[3] - q[1]));
        box[4 * i] = ix0;
        box[4 * i + 1] = ix1;
        box[4 * i + 2] = iy0;
        box[4 * i + 3] = iy1;
    }
    // Pixel (x, y) -- widened by kCamBinMargin -- against triangle i beyond its box: separated when all
    // four corners lie strictly outside one of its projected edges (the separating-axis test of a
    // triangle and a square; the box test is the square's own axes). Projections of (nearly) zero
    // area keep the whole box.
    auto meets = [&](size_t i, int x, int y) {
        const double A = parea[i];
        if (!(std::fabs(A) > 1e-6)) return true;
        const double *q = &q2[6 * i];
        const double sg = A > 0.0 ? 1.0 : -1.0;
        const double cx[4] = {x - kCamBinMargin, x + 1 + kCamBinMargin, x - kCamBinMargin, x + 1 + kCamBinMargin};
        const double cy[4] = {y - kCamBinMargin, y - kCamBinMargin, y + 1 + kCamBinMargin, y + 1 + kCamBinMargin};
        for (int e = 0; e < 3; ++e) {
            const double ax = q[2 * e], ay = q[2 * e + 1];
            const double bx = q[2 * ((e + 1) % 3)], by = q[2 * ((e + 1) % 3) + 1];
            bool all_out = true;
            for (int k = 0; k < 4 && all_out; ++k)
                all_out = sg * ((bx - ax) * (cy[k] - ay) - (by - ay) * (cx[k] - ax)) < 0.0;
            if (all_out) return false;
        }
        return true;
    };
    for (size_t i = 0; i < n; ++i) {
        if (tag[i] == kAll) b.all.push_back((int32_t)i);
        if (tag[i] != kBox) continue;
        for (int y = box[4 * i + 2]; y <= box[4 * i + 3]; ++y)
            for (int x = box[4 * i]; x <= box[4 * i + 1]; ++x)
                if (meets(i, x, y)) ++b.off[(size_t)y * b.w + x + 1];
    }
    for (size_t p = 1; p < b.off.size(); ++p) b.off[p] += b.off[p - 1];
    b.tri.resize(b.off.back());
    std::vector<uint32_t> cur(b.off.begin(), b.off.end() - 1);
    for (size_t i = 0; i < n; ++i) {
        if (tag[i] != kBox) continue;
        for (int y = box[4 * i + 2]; y <= box[4 * i + 3]; ++y)
            for (int x = box[4 * i]; x <= box[4 * i + 1]; ++x)
                if (meets(i, x, y)) b.tri[cur[(size_t)y * b.w + x]++] = (int32_t)i;
    }
    // each pixel's list by projected area, largest first: a camera ray stops at its first hit, and the
    // wave once every lane has one, so the triangles covering most of the pixel go first (the answer
    // does not depend on the order)
    for (size_t p = 0; p + 1 < b.off.size(); ++p)
        if (b.off[p + 1] - b.off[p] > 1)
            std::stable_sort(b.tri.begin() + b.off[p], b.tri.begin() + b.off[p + 1],
                             [&](int32_t u, int32_t v) { return std::fabs(parea[u]) > std::fabs(parea[v]); });
}

}  // namespace mpss
