// bvh_sah.h — the non-parity fast BVH, host code.
//
// The reference builds its BVH by a median split on the longest axis with an inconsistent
// comparator (BVHNode.java:13-69) and walks it right child first with no near-first order
// (compute.glsl:226-266): scene 8 costs 77.8 node visits and 11.7 primitive tests per sample.
// This builder makes a binned-SAH tree over the same primitives, in the reference's own
// node format (rt_bvh_node, BVHNode.java:47-56), so that everything downstream is unchanged:
// the threaded / link-format walk, the kernel, the LDS plan, the spine entry, and the CPU
// oracle (which walks any BVH in this format, so the kernel stays bit-exact against the
// oracle *on the SAH tree*).  Against the reference BVH it is not bit-exact: a medium's
// rand() draws happen at another point of the visit sequence (and exact ties resolve by
// another order), so images agree statistically, not bit for bit (tests/test_gpu_fast_bvh.py).
//
// What is preserved so that the statistics match the reference's:
//   * the primitive set: exactly the prims the uploaded BVH's leaves reference;
//   * each medium's test multiplicity: a medium in a singleton leaf of the reference BVH is
//     tested twice per walk (BVHNode.java:33-34) -- which doubles its
//     effective density -- and stays a singleton leaf here; a medium in a two-prim leaf
//     keeps that leaf (same partner, same order) as one unit, tested once;
//   * leaves of at most two prims (the format's two child slots).
// Child order: the reference pops the right child first; here the child whose box centre is
// nearer the camera is made the right child (visited first).  The oracle's counters on scene 8
// (240x135, 8 frames, depth 5; profiles/r05_sah_orders.log): reference BVH 77.5 node visits and
// 7.6 solid + medium tests per sample; SAH larger-first 41.0 / 6.8, smaller-first 39.2 / 6.8,
// camera-nearer-first 35.5 / 6.0.  Leaf cost 1 node step per prim test (more pair leaves, 1867
// nodes; 2, 4, 8 give 2627-2809 nodes of mostly singleton leaves at the same visit counts).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "rt/rt_types.h"

namespace rt_sah {

struct Box3 {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float p[3]) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void join(const Box3& b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    bool valid() const { return lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]; }
    double area() const {
        if (!valid()) return 0.0;
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

// One unit of the build: a solo prim, or a fixed leaf (a medium with its reference partner,
// or a medium tested twice) that is never split.
struct Item {
    Box3 b;
    float c[3];
    int32_t a, b_id;   // packed ids (index << 16 | type); b_id = a for a singleton
    bool fixed;        // a whole leaf already
    int prims() const { return fixed && a != b_id ? 2 : 1; }
};

inline int32_t pack(int type, int idx) { return (int32_t)(((uint32_t)idx << 16) | (uint32_t)(type & 0xFFFF)); }

struct Input {
    const rt_sphere* sph = nullptr; size_t n_sph = 0;
    const rt_quad* quad = nullptr; size_t n_quad = 0;
    const rt_medium* med = nullptr; size_t n_med = 0;
    const rt_box* box = nullptr; size_t n_box = 0;
    const rt_bvh_node* ref = nullptr; size_t n_ref = 0;
};

inline void quad_box(const rt_quad& q, Box3& b) {
    float p[3];
    for (int s = 0; s < 4; s++) {
        for (int k = 0; k < 3; k++) p[k] = q.q[k] + ((s & 1) ? q.u[k] : 0.0f) + ((s & 2) ? q.v[k] : 0.0f);
        b.grow(p);
    }
}

// AABB of a prim (Sphere / Quad / Box / ConstantMedium.java bounding boxes), padded to the
// reference's 0.001 minimum thickness (AABB.java:59-64) and grown by a relative 2^-20 so that a
// hit the float prim test accepts is never outside its box.  false: a missing record.
inline bool prim_box(const Input& in, int type, int idx, Box3& b, int depth = 0) {
    b = Box3();
    if (idx < 0) return false;
    if (type == RT_MODEL_SPHERE) {
        if ((size_t)idx >= in.n_sph) return false;
        const rt_sphere& s = in.sph[idx];
        const float r = std::fabs(s.radius);
        float p[3];
        for (int e = 0; e < 2; e++)
            for (int sg = -1; sg <= 1; sg += 2) {
                for (int k = 0; k < 3; k++) p[k] = s.center1[k] + (e ? s.center_vec[k] : 0.0f) + sg * r;
                b.grow(p);
            }
    } else if (type == RT_MODEL_QUAD) {
        if ((size_t)idx >= in.n_quad) return false;
        quad_box(in.quad[idx], b);
    } else if (type == RT_MODEL_BOX) {
        if ((size_t)idx >= in.n_box) return false;
        for (int f = 0; f < 6; f++) quad_box(in.box[idx].quads[f], b);
    } else if (type == RT_MODEL_CONSTANT_MEDIUM) {
        if ((size_t)idx >= in.n_med || depth > 0) return false;
        return prim_box(in, in.med[idx].boundary_type, in.med[idx].boundary_idx, b, 1);
    } else {
        return false;
    }
    for (int k = 0; k < 3; k++) {
        if (!(b.lo[k] <= b.hi[k])) return false;   // NaN
        if (b.hi[k] - b.lo[k] < 0.001f) {
            const float m = 0.0005f;
            b.lo[k] -= m;
            b.hi[k] += m;
        }
        const float g = (std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])) + 1.0f) * 0x1p-20f;
        b.lo[k] -= g;
        b.hi[k] += g;
    }
    return true;
}

class Builder {
public:
    // order: 0 = larger surface area visited first, 1 = smaller first, 2 = nearer to `eye`
    // first (rt_set_bvh_mode's, with the camera position)
    Builder(const Input& in, int order, const float eye[3], double prim_cost = 1.0)
        : in_(in), order_(order), kPrim(prim_cost) {
        for (int k = 0; k < 3; k++) eye_[k] = eye ? eye[k] : 0.0f;
    }

    // false: the reference BVH references a missing record or is empty
    bool build(std::vector<rt_bvh_node>& out) {
        out.clear();
        if (!collect()) return false;
        if (items_.empty()) return false;
        nodes_.clear();
        std::vector<int> ids(items_.size());
        for (size_t i = 0; i < ids.size(); i++) ids[i] = (int)i;
        node(ids, 0, (int)ids.size(), 1);
        out.swap(nodes_);
        return true;
    }

private:
    const Input& in_;
    int order_;
    const double kPrim;   // SAH cost of a prim test in node steps (a leaf test costs several in the kernel)
    float eye_[3];
    std::vector<Item> items_;
    std::vector<rt_bvh_node> nodes_;
    static constexpr double kNode = 1.0;
    static constexpr int kBins = 32;

    bool item_of(int32_t a, int32_t b, bool fixed, Item& it) {
        Box3 ba, bb;
        if (!prim_box(in_, a & 0xFFFF, (int)((uint32_t)a >> 16), ba)) return false;
        if (!prim_box(in_, b & 0xFFFF, (int)((uint32_t)b >> 16), bb)) return false;
        it.b = ba;
        it.b.join(bb);
        for (int k = 0; k < 3; k++) it.c[k] = 0.5f * (it.b.lo[k] + it.b.hi[k]);
        it.a = a;
        it.b_id = b;
        it.fixed = fixed;
        return true;
    }

    // the prims of the reference BVH's leaves: media keep their leaf, the rest become solo items
    bool collect() {
        items_.clear();
        std::map<int32_t, bool> seen;
        for (size_t i = 0; i < in_.n_ref; i++) {
            const rt_bvh_node& n = in_.ref[i];
            const int lt = n.left_id & 0xFFFF, rt = n.right_id & 0xFFFF;
            if (lt == 0 && rt == 0) continue;   // inner node
            if (lt == 0 || rt == 0) return false;   // a mixed node: not the reference's format
            const bool med = lt == RT_MODEL_CONSTANT_MEDIUM || rt == RT_MODEL_CONSTANT_MEDIUM;
            if (med) {
                if (seen.count(n.left_id) || seen.count(n.right_id)) return false;
                Item it;
                if (!item_of(n.left_id, n.right_id, true, it)) return false;
                items_.push_back(it);
                seen[n.left_id] = seen[n.right_id] = true;
                continue;
            }
            for (int32_t p : {n.left_id, n.right_id}) {
                if (seen.count(p)) continue;
                Item it;
                if (!item_of(p, p, false, it)) return false;
                items_.push_back(it);
                seen[p] = true;
            }
        }
        return true;
    }

    Box3 bounds(const std::vector<int>& ids, int s, int e) const {
        Box3 b;
        for (int i = s; i < e; i++) b.join(items_[ids[i]].b);
        return b;
    }
    int prims(const std::vector<int>& ids, int s, int e) const {
        int n = 0;
        for (int i = s; i < e; i++) n += items_[ids[i]].prims();
        return n;
    }

    int emit() {
        nodes_.push_back(rt_bvh_node());
        return (int)nodes_.size() - 1;
    }
    void set_box(int at, const Box3& b) {
        rt_bvh_node& n = nodes_[at];
        n.xmin = b.lo[0]; n.xmax = b.hi[0]; n.ymin = b.lo[1]; n.ymax = b.hi[1]; n.zmin = b.lo[2]; n.zmax = b.hi[2];
    }

    // a leaf node: its left prim is tested first, then its right (compute.glsl:247-256)
    int leaf(int32_t first, int32_t second, const Box3& b) {
        const int at = emit();
        set_box(at, b);
        nodes_[at].left_id = first;
        nodes_[at].right_id = second;
        return at;
    }

    // is child box A visited before B?
    bool first(const Box3& a, const Box3& b) const {
        if (order_ == 2) {
            auto d2 = [&](const Box3& x) {
                double s = 0;
                for (int k = 0; k < 3; k++) {
                    const double c = 0.5 * ((double)x.lo[k] + x.hi[k]) - eye_[k];
                    s += c * c;
                }
                return s;
            };
            return d2(a) <= d2(b);
        }
        return order_ == 1 ? a.area() <= b.area() : a.area() >= b.area();
    }

    int node(std::vector<int>& ids, int s, int e, int depth) {
        const int n = e - s;
        const Box3 bb = bounds(ids, s, e);
        if (n == 1) {
            const Item& it = items_[ids[s]];
            // a fixed leaf keeps the reference's (left, right)
            if (it.fixed) return leaf(it.a, it.b_id, bb);
            return leaf(it.a, it.a, bb);
        }
        if (n == 2 && !items_[ids[s]].fixed && !items_[ids[s + 1]].fixed) {
            // one leaf of two prims, or two singleton leaves under a node
            const Box3 b0 = items_[ids[s]].b, b1 = items_[ids[s + 1]].b;
            const double pa = std::max(bb.area(), 1e-30);
            const double split = kNode + kPrim * (b0.area() + b1.area()) / pa;
            if (2.0 * kPrim <= split) {
                const bool f0 = first(b0, b1);
                return leaf(items_[ids[s + (f0 ? 0 : 1)]].a, items_[ids[s + (f0 ? 1 : 0)]].a, bb);
            }
        }
        int mid = s + n / 2;
        if (depth < 40) mid = sah_split(ids, s, e, bb);
        if (mid <= s || mid >= e) {   // degenerate: median on the longest centroid axis
            Box3 cb;
            for (int i = s; i < e; i++) cb.grow(items_[ids[i]].c);
            int ax = 0;
            for (int k = 1; k < 3; k++)
                if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
            mid = s + n / 2;
            std::nth_element(ids.begin() + s, ids.begin() + mid, ids.begin() + e,
                             [&](int x, int y) { return items_[x].c[ax] < items_[y].c[ax]; });
        }
        const int at = emit();
        set_box(at, bb);
        const Box3 bl = bounds(ids, s, mid), br = bounds(ids, mid, e);
        const bool l_first = first(bl, br);
        int c0 = node(ids, s, mid, depth + 1);
        int c1 = node(ids, mid, e, depth + 1);
        // right = visited first
        nodes_[at].right_id = pack(RT_MODEL_BVH_NODE, l_first ? c0 : c1);
        nodes_[at].left_id = pack(RT_MODEL_BVH_NODE, l_first ? c1 : c0);
        return at;
    }

    // binned SAH over the item centroids; returns the split position after partitioning ids
    int sah_split(std::vector<int>& ids, int s, int e, const Box3& bb) {
        Box3 cb;
        for (int i = s; i < e; i++) cb.grow(items_[ids[i]].c);
        const double pa = std::max(bb.area(), 1e-30);
        double best = INFINITY;
        int best_ax = -1, best_bin = -1;
        for (int ax = 0; ax < 3; ax++) {
            const float lo = cb.lo[ax], ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.0f)) continue;
            Box3 bx[kBins];
            int cnt[kBins] = {};
            auto bin = [&](const Item& it) {   // a non-finite centroid (NaN, inf) goes to an end bin
                const float f = (it.c[ax] - lo) / ext * kBins;
                return f >= (float)kBins ? kBins - 1 : (f >= 0.0f ? (int)f : 0);
            };
            for (int i = s; i < e; i++) {
                const Item& it = items_[ids[i]];
                const int k = bin(it);
                bx[k].join(it.b);
                cnt[k] += it.prims();
            }
            double ra[kBins];
            int rc[kBins];
            Box3 acc;
            int c = 0;
            for (int k = kBins - 1; k > 0; k--) {
                acc.join(bx[k]);
                c += cnt[k];
                ra[k] = acc.area();
                rc[k] = c;
            }
            Box3 la;
            int lc = 0;
            for (int k = 0; k < kBins - 1; k++) {
                la.join(bx[k]);
                lc += cnt[k];
                if (lc == 0 || rc[k + 1] == 0) continue;
                const double cost = kNode + kPrim * (la.area() * lc + ra[k + 1] * rc[k + 1]) / pa;
                if (cost < best) {
                    best = cost;
                    best_ax = ax;
                    best_bin = k;
                }
            }
        }
        if (best_ax < 0) return s;
        const float lo = cb.lo[best_ax], ext = cb.hi[best_ax] - cb.lo[best_ax];
        auto left = [&](int id) {   // the bins of sah_split's count (a non-finite centroid: an end bin)
            const float f = (items_[id].c[best_ax] - lo) / ext * kBins;
            return (f >= (float)kBins ? kBins - 1 : (f >= 0.0f ? (int)f : 0)) <= best_bin;
        };
        return (int)(std::stable_partition(ids.begin() + s, ids.begin() + e, left) - ids.begin());
    }
};

}  // namespace rt_sah
