// rrt_host.cpp — host runtime of librrt_hip.so: the C-ABI of include/rrt_hip.h.
//
//   scene builder     == gpu::build_in_one_weekend_scene   (src/gpu/mod.rs:124-301)
//   BVH build         binned SAH per BvhNode::build       (src/books/in_one_weekend/bvh.rs:21-156)
//   one-shot render   replaces cuda::imp::render          (src/cuda/mod.rs:342-439)
//   PPM writer        == render_io::write_ppm_from_accum  (src/render_io.rs:3-31)
//
// Device memory is owned by RrtScene; the one-shot entry frees everything before it
// returns (ownership contract of SURVEY §8b). No CPU rendering fallback exists here:
// without a HIP device every render entry fails with RRT_E_NODEV.
#include "rrt_internal.h"
#include "../../include/rrt_hip.h"

#include <algorithm>
#include <limits>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr, what)                                                                   \
    do {                                                                                      \
        hipError_t e__ = (expr);                                                              \
        if (e__ != hipSuccess)                                                                \
            return fail(RRT_E_HIP, std::string(what) + " failed: " + hipGetErrorString(e__)); \
    } while (0)

// ------------------------------------------------------------------------------------
// rand 0.8.5 SmallRng (= Xoshiro256++ on 64-bit) with seed_from_u64's SplitMix64 fill,
// and the Standard / UniformFloat float conversions it applies (Cargo.lock:810-812).
// Restated from the published algorithms (the crate is not in this image: unpinned).
// ------------------------------------------------------------------------------------
struct SmallRng {
    uint64_t s[4];
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    explicit SmallRng(uint64_t state) {
        const uint64_t phi = 0x9e3779b97f4a7c15ull;
        for (int i = 0; i < 4; ++i) {
            state += phi;
            uint64_t z = state;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            s[i] = z ^ (z >> 31);
        }
    }
    uint64_t next_u64() {
        const uint64_t result = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return result;
    }
    uint32_t next_u32() { return (uint32_t)(next_u64() >> 32); }
    float gen_f32() { return (float)(next_u32() >> 8) * (1.0f / 16777216.0f); }          // Standard f32
    double gen_f64() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }  // Standard f64
    double gen_range_f64(double lo, double hi) {  // UniformFloat<f64>::sample_single
        const double scale = hi - lo;
        for (;;) {
            const uint64_t bits = (next_u64() >> 12) | (1023ull << 52);
            double v12;
            std::memcpy(&v12, &bits, 8);
            const double res = (v12 - 1.0) * scale + lo;
            if (res < hi) return res;
        }
    }
    float gen_range_f32(float lo, float hi) {  // UniformFloat<f32>::sample_single
        const float scale = hi - lo;
        for (;;) {
            uint32_t bits = (next_u32() >> 9) | (127u << 23);
            float v12;
            std::memcpy(&v12, &bits, 4);
            const float res = (v12 - 1.0f) * scale + lo;
            if (res < hi) return res;
        }
    }
};

struct D3 {
    double x, y, z;
};
D3 d3(double x, double y, double z) { return D3{x, y, z}; }
D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
D3 operator*(D3 a, double s) { return d3(a.x * s, a.y * s, a.z * s); }
D3 operator/(D3 a, double s) { return d3(a.x / s, a.y / s, a.z / s); }  // gpu/mod.rs:89-95 divides
double length(D3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
D3 cross(D3 a, D3 b) { return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
D3 unit_vector(D3 v) { return v / length(v); }
double degrees_to_radians(double deg) { return deg * M_PI / 180.0; }

void put4(float *dst, float a, float b, float c, float d) {
    dst[0] = a;
    dst[1] = b;
    dst[2] = c;
    dst[3] = d;
}

// ------------------------------------------------------------------------------------
// BVH over the sphere boxes (aabb.rs padding, sphere.rs:16-21 bounds): by default a full
// sweep SAH on all three axes (Builder::sweep); RRT_BVH_SPLIT=binned selects the reference's
// own criterion — binned SAH exactly as bvh.rs:21-156 chooses splits (12 buckets, longest axis
// of the node bbox, stable-sort+median fallbacks). Leaves hold <= max_leaf spheres; the tree
// is flattened into GNodes (80 B in LDS, 32 B in global memory) with both child boxes in the parent. The tree only changes
// which boxes are tested, never a sphere's result.
// ------------------------------------------------------------------------------------
struct Interval {
    double min, max;
    double size() const { return max - min; }
};
struct Aabb {
    Interval ax[3];
};
const double kInf = std::numeric_limits<double>::infinity();

Interval iv_union(Interval a, Interval b) {  // interval.rs:44-49
    return Interval{a.min <= b.min ? a.min : b.min, a.max >= b.max ? a.max : b.max};
}
Aabb pad(Aabb b) {  // aabb.rs:104-115
    const double delta = 0.0001;
    for (int i = 0; i < 3; ++i)
        if (b.ax[i].size() < delta) b.ax[i] = Interval{b.ax[i].min - delta / 2.0, b.ax[i].max + delta / 2.0};
    return b;
}
Aabb aabb_empty() { return Aabb{{{kInf, -kInf}, {kInf, -kInf}, {kInf, -kInf}}}; }
Aabb aabb_union(const Aabb &a, const Aabb &b) {
    return pad(Aabb{{iv_union(a.ax[0], b.ax[0]), iv_union(a.ax[1], b.ax[1]), iv_union(a.ax[2], b.ax[2])}});
}
int longest_axis(const Aabb &b) {  // aabb.rs:87-95
    if (b.ax[0].size() > b.ax[1].size()) return b.ax[0].size() > b.ax[2].size() ? 0 : 2;
    return b.ax[1].size() > b.ax[2].size() ? 1 : 2;
}
double surface_area(const Aabb &b) {
    const double a = b.ax[0].size(), c1 = b.ax[1].size(), c2 = b.ax[2].size();
    return 2.0 * (a * c1 + a * c2 + c1 * c2);
}

float f32_down(double d) {
    float f = (float)d;
    if ((double)f > d) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}
float f32_up(double d) {
    float f = (float)d;
    if ((double)f < d) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

struct Builder {
    const std::vector<Aabb> &boxes;
    std::vector<uint32_t> objs;
    uint32_t max_leaf;
    // Split criterion: false = bvh.rs's (12 buckets on the longest axis); true (default) = full
    // sweep SAH over sorted centroids on all three axes, with small nodes kept as leaves unless
    // splitting is cheaper: leaf cost n (sphere tests) vs node_cost + (A_l n_l + A_r n_r)/A.
    // node_cost 2 (a node visit ~ two sphere tests in this kernel) measured best: C2 +3.5 %
    // over the bvh.rs criterion, and the RTOW tree (203 nodes) still fits the LDS budget.
    bool sweep = true;
    double node_cost = 2.0;  // kNodeCost (f32 kernel) or f64_node_cost() (f64 kernel), set by build_bvh

    // Binary SAH tree (bvh.rs:16-156 split choice), leaves of <= max_leaf spheres.
    struct BNode {
        Aabb box;
        int32_t left = -1, right = -1;  // children (internal)
        int32_t first = 0, count = 0;   // primitive range (leaf)
        bool leaf = false;
    };
    std::vector<BNode> bin;

    Builder(const std::vector<Aabb> &b, uint32_t leaf) : boxes(b), max_leaf(leaf) {
        objs.resize(b.size());
        for (size_t i = 0; i < b.size(); ++i) objs[i] = (uint32_t)i;
    }

    double centroid(uint32_t o, int axis) const {
        return 0.5 * (boxes[o].ax[axis].min + boxes[o].ax[axis].max);
    }

    void sort_by_min(size_t lo, size_t hi, int axis) {  // Rust slice::sort_by is stable
        std::stable_sort(objs.begin() + lo, objs.begin() + hi, [&](uint32_t a, uint32_t b) {
            return boxes[a].ax[axis].min < boxes[b].ax[axis].min;
        });
    }

    // bvh.rs:34-152: returns the split point (absolute index) for objs[lo, hi)
    size_t split(size_t lo, size_t hi, const Aabb &bbox) {
        const size_t span = hi - lo;
        constexpr int kBuckets = 12;
        const int axis = longest_axis(bbox);
        double cmin = kInf, cmax = -kInf;
        for (size_t i = lo; i < hi; ++i) {
            const double c = centroid(objs[i], axis);
            if (c < cmin) cmin = c;
            if (c > cmax) cmax = c;
        }
        if (std::fabs(cmax - cmin) < 1e-12) {
            sort_by_min(lo, hi, axis);
            return lo + span / 2;
        }
        auto bucket_of = [&](uint32_t o) {
            size_t idx = (size_t)((centroid(o, axis) - cmin) / (cmax - cmin) * (double)kBuckets);
            return idx >= (size_t)kBuckets ? (size_t)kBuckets - 1 : idx;
        };
        size_t count[kBuckets] = {0};
        Aabb bb[kBuckets];
        for (int i = 0; i < kBuckets; ++i) bb[i] = aabb_empty();
        for (size_t i = lo; i < hi; ++i) {
            const size_t b = bucket_of(objs[i]);
            count[b]++;
            bb[b] = aabb_union(bb[b], boxes[objs[i]]);
        }
        Aabb right_bb[kBuckets];
        size_t right_cnt[kBuckets];
        Aabb acc = aabb_empty();
        size_t acc_n = 0;
        for (int i = kBuckets - 1; i >= 0; --i) {
            acc_n += count[i];
            acc = aabb_union(acc, bb[i]);
            right_bb[i] = acc;
            right_cnt[i] = acc_n;
        }
        Aabb left = aabb_empty();
        size_t left_n = 0;
        double best = kInf;
        size_t best_split = 0;
        for (int i = 0; i < kBuckets - 1; ++i) {
            left_n += count[i];
            left = aabb_union(left, bb[i]);
            if (left_n == 0 || right_cnt[i + 1] == 0) continue;
            const double cost = surface_area(left) * (double)left_n + surface_area(right_bb[i + 1]) * (double)right_cnt[i + 1];
            if (cost < best) {
                best = cost;
                best_split = (size_t)i;
            }
        }
        if (!std::isfinite(best)) {
            sort_by_min(lo, hi, axis);
            return lo + span / 2;
        }
        size_t mid = 0;
        for (size_t i = 0; i < span; ++i) {
            if (bucket_of(objs[lo + i]) <= best_split) {
                std::swap(objs[lo + i], objs[lo + mid]);
                ++mid;
            }
        }
        if (mid == 0 || mid == span) {
            sort_by_min(lo, hi, axis);
            return lo + span / 2;
        }
        return lo + mid;
    }

    // Exact SAH sweep: best (axis, position) over centroid-sorted orders of objs[lo, hi);
    // reorders objs[lo, hi) into the winning order and returns (split index, A_l n_l + A_r n_r).
    size_t split_sweep(size_t lo, size_t hi, double &best_cost) {
        const size_t n = hi - lo;
        std::vector<uint32_t> order[3];
        std::vector<double> right_area(n + 1);
        best_cost = kInf;
        int best_axis = 0;
        size_t best_i = n / 2;
        for (int axis = 0; axis < 3; ++axis) {
            order[axis].assign(objs.begin() + lo, objs.begin() + hi);
            std::stable_sort(order[axis].begin(), order[axis].end(), [&](uint32_t a, uint32_t b) {
                return centroid(a, axis) < centroid(b, axis);
            });
            Aabb acc = aabb_empty();
            for (size_t i = n; i-- > 1;) {
                acc = aabb_union(acc, boxes[order[axis][i]]);
                right_area[i] = surface_area(acc);
            }
            acc = aabb_empty();
            for (size_t i = 1; i < n; ++i) {
                acc = aabb_union(acc, boxes[order[axis][i - 1]]);
                const double cost = surface_area(acc) * (double)i + right_area[i] * (double)(n - i);
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_i = i;
                }
            }
        }
        std::copy(order[best_axis].begin(), order[best_axis].end(), objs.begin() + lo);
        return lo + best_i;
    }

    int32_t build(size_t lo, size_t hi) {
        Aabb bbox = aabb_empty();
        for (size_t i = lo; i < hi; ++i) bbox = aabb_union(bbox, boxes[objs[i]]);
        const int32_t me = (int32_t)bin.size();
        bin.push_back(BNode{});
        bin[me].box = bbox;
        const size_t span = hi - lo;
        size_t mid;
        if (sweep && span > 1) {
            double cost = kInf;
            mid = split_sweep(lo, hi, cost);
            const double area = surface_area(bbox);
            const bool keep_leaf = span <= max_leaf && !(area > 0.0 && node_cost + cost / area < (double)span);
            if (keep_leaf) {
                bin[me].leaf = true;
                bin[me].first = (int32_t)lo;
                bin[me].count = (int32_t)span;
                return me;
            }
        } else if (span <= max_leaf) {
            bin[me].leaf = true;
            bin[me].first = (int32_t)lo;
            bin[me].count = (int32_t)span;
            return me;
        } else {
            mid = split(lo, hi, bbox);
        }
        const int32_t l = build(lo, mid);
        const int32_t r = build(mid, hi);
        bin[me].left = l;
        bin[me].right = r;
        return me;
    }
};

// Flattened device BVH (either width) plus the numbers the kernel needs.
struct FlatBvh {
    std::vector<uint8_t> bytes;
    uint32_t n_nodes = 0, n_leaves = 0, max_depth = 0, max_leaf = 0, stack_need = 0, width = 2;
    uint32_t stride = 0;  // bytes per node: 80 (BVH2, sign-ordered, LDS), 32 (BVH2, f16, global), 128 (BVH4)
    // BVH2: every node whose children are both leaves has them adjacent in primitive order
    // (right.first == left.first + left.count), so the kernel tests the hit ones as one range
    bool sibling_leaves_adjacent = true;
    // Unbounded media: sphere-bounded media whose box holds every other primitive's (a fog around
    // the whole scene, the_next_week/mod.rs:563-566). Every ray's box test would pass them, so they
    // are not in the tree: they follow its primitives in leaf order (the last n_unbounded entries)
    // and each closest-hit query tests them after the walk, every lane of the wave together.
    uint32_t n_unbounded = 0;
};

// Conservative slab test in f32. The kernel's plane distance fma(P, inv, -o*inv) differs from
// the exact (P - o)/d by at most u(2|P - o| + |o|)/|d| along axis a (u = 2^-24: the roundings
// of 1/d, of o*inv and of the fma), and the primitive tests' own t carry a few ulps. Growing
// each stored box face by 4u(2|P| + 3 O_a) in position space — O_a = the largest |coordinate|
// on axis a of the scene's bounds, which holds every ray origin (hit points, and cameras inside
// the scene's extent) — covers all of it, so a box never rejects a ray its primitives would hit
// (a missed grazing hit at final_scene's |p| ~ 2000 showed the need). The growth is ~1e-5 of
// a box's size at RTOW scale; traversal cost unchanged within noise.
struct BoxSlack {
    double o[3] = {0.0, 0.0, 0.0};
    explicit BoxSlack(const Aabb &scene) {
        for (int a = 0; a < 3; ++a) {
            const double m = std::max(std::fabs(scene.ax[a].min), std::fabs(scene.ax[a].max));
            if (std::isfinite(m) && m < 1e29) o[a] = m;
        }
    }
    double grow(int a, double p) const { return 4.0 * 0x1.0p-24 * (2.0 * std::fabs(p) + 3.0 * o[a]); }
};

void put_box(float *lo, float *hi, const Aabb &b, const BoxSlack *slack) {
    for (int a = 0; a < 3; ++a) {
        double mn = b.ax[a].min, mx = b.ax[a].max;
        if (slack && mn <= mx && std::isfinite(mn) && std::isfinite(mx) && mx < 1e29) {
            mn -= slack->grow(a, mn);
            mx += slack->grow(a, mx);
        }
        lo[a] = f32_down(mn);
        hi[a] = f32_up(mx);
    }
}

// A child slot no ray can enter: a point box at 1e30 (rejected for every direction,
// including zero components where the slab test produces +-inf).
Aabb never_hit_box() {
    Aabb b;
    for (int i = 0; i < 3; ++i) b.ax[i] = Interval{1e30, 1e30};
    return b;
}

void put_node2(rrt::GNode &n, const float *lo0, const float *hi0, const float *lo1, const float *hi1, int32_t ref0,
               int32_t cnt0, int32_t ref1, int32_t cnt1) {
    const float *lo[2] = {lo0, lo1}, *hi[2] = {hi0, hi1};
    for (int c = 0; c < 2; ++c)
        for (int a = 0; a < 3; ++a) {
            n.box[c][3 * a] = lo[c][a];
            n.box[c][3 * a + 1] = hi[c][a];
            n.box[c][3 * a + 2] = lo[c][a];
        }
    n.link[0] = (uint32_t)ref0 | ((uint32_t)cnt0 << rrt::kLinkCountShift);
    n.link[1] = (uint32_t)ref1 | ((uint32_t)cnt1 << rrt::kLinkCountShift);
}

// f32 -> f16 bits rounded toward -inf (down) or +inf (up); a subnormal result is pushed outward to
// 0 or the smallest normal, so the kernel never reads an f16 subnormal plane.
uint16_t f16_bits(float x) {
    const _Float16 h = (_Float16)x;
    uint16_t b;
    std::memcpy(&b, &h, 2);
    return b;
}
float f16_value(uint16_t b) {
    _Float16 h;
    std::memcpy(&h, &b, 2);
    return (float)h;
}
uint16_t f16_round(float x, bool up) {
    uint16_t b = f16_bits(x);
    const float v = f16_value(b);
    if (up ? v < x : v > x) {  // one f16 step outward (toward +inf / -inf)
        if ((b & 0x7fffu) == 0) b = up ? 0x0001u : 0x8001u;
        else if (((b & 0x8000u) != 0) == up) b = (uint16_t)(b - 1u);
        else b = (uint16_t)(b + 1u);
    }
    if ((b & 0x7c00u) == 0 && (b & 0x03ffu) != 0) {  // subnormal: outward to 0 or +-2^-14
        const bool neg = (b & 0x8000u) != 0;
        b = up ? (neg ? 0x8000u : 0x0400u) : (neg ? 0x8400u : 0x0000u);
    }
    return b;
}
void put_node2(rrt::GNodeH &n, const float *lo0, const float *hi0, const float *lo1, const float *hi1, int32_t ref0,
               int32_t cnt0, int32_t ref1, int32_t cnt1) {
    const float *lo[2] = {lo0, lo1}, *hi[2] = {hi0, hi1};
    uint32_t *dst[2] = {n.c0, n.c1};
    for (int c = 0; c < 2; ++c) {
        const bool never = lo[c][0] >= 1e30f;  // never_hit_box(): the point (65504, 65504, 65504)
        for (int a = 0; a < 3; ++a) {
            const uint16_t l = never ? 0x7bffu : f16_round(lo[c][a], false);
            const uint16_t h = never ? 0x7bffu : f16_round(hi[c][a], true);
            dst[c][a] = (uint32_t)l | ((uint32_t)h << 16);
        }
    }
    n.link[0] = (uint32_t)ref0 | ((uint32_t)cnt0 << rrt::kLinkCountShift);
    n.link[1] = (uint32_t)ref1 | ((uint32_t)cnt1 << rrt::kLinkCountShift);
}

// BVH2: the binary tree as is, root = node 0, both child boxes stored in the parent; Node =
// rrt::GNode (80 B, sign-ordered planes, LDS) or rrt::GNodeH (32 B, f16 planes, global memory).
template <class Node>
FlatBvh flatten2(const Builder &bd, int32_t root) {
    FlatBvh f;
    const BoxSlack slack(bd.bin[root].box);
    std::vector<Node> out;
    struct Item { int32_t bin; int32_t slot; };
    auto child_ref = [&](int32_t c, float *lo, float *hi, int32_t &ref, int32_t &cnt, std::vector<Item> &todo) {
        const Builder::BNode &b = bd.bin[c];
        put_box(lo, hi, b.leaf && b.count == 0 ? never_hit_box() : b.box, &slack);
        if (b.leaf) {
            ref = b.first;
            cnt = b.count;
            f.n_leaves++;
            f.max_leaf = std::max<uint32_t>(f.max_leaf, (uint32_t)b.count);
        } else {
            ref = (int32_t)out.size();
            cnt = 0;
            out.push_back(Node{});
            todo.push_back(Item{c, ref});
        }
    };
    std::vector<std::pair<Item, uint32_t>> stack;  // (item, depth)
    out.push_back(Node{});
    std::vector<Item> todo;
    const Builder::BNode &r = bd.bin[root];
    if (r.leaf) {  // whole scene in one leaf: child 0 = the leaf, child 1 = never hit
        float lo0[3], hi0[3], lo1[3], hi1[3];
        int32_t ref0, cnt0;
        child_ref(root, lo0, hi0, ref0, cnt0, todo);
        put_box(lo1, hi1, never_hit_box(), nullptr);
        put_node2(out[0], lo0, hi0, lo1, hi1, ref0, cnt0, 0, 0);
        f.max_depth = 1;
    } else {
        stack.push_back({Item{root, 0}, 0});
        while (!stack.empty()) {
            auto [it, depth] = stack.back();
            stack.pop_back();
            f.max_depth = std::max(f.max_depth, depth + 1);
            const Builder::BNode &b = bd.bin[it.bin];
            float lo0[3], hi0[3], lo1[3], hi1[3];
            int32_t ref0, cnt0, ref1, cnt1;
            todo.clear();
            child_ref(b.left, lo0, hi0, ref0, cnt0, todo);
            child_ref(b.right, lo1, hi1, ref1, cnt1, todo);
            if (cnt0 > 0 && cnt1 > 0 && ref1 != ref0 + cnt0) f.sibling_leaves_adjacent = false;
            put_node2(out[it.slot], lo0, hi0, lo1, hi1, ref0, cnt0, ref1, cnt1);
            for (auto &t : todo) stack.push_back({t, depth + 1});
        }
    }
    f.n_nodes = (uint32_t)out.size();
    f.stack_need = f.max_depth + 1;
    f.width = 2;
    f.stride = (uint32_t)sizeof(Node);
    f.bytes.resize(out.size() * sizeof(Node));
    std::memcpy(f.bytes.data(), out.data(), f.bytes.size());
    return f;
}

// BVH4: collapse the binary tree — each wide node adopts up to 4 descendants, repeatedly
// opening the internal candidate with the largest surface area (the standard SAH-guided
// collapse). Empty slots get the never-hit box.
FlatBvh flatten4(const Builder &bd, int32_t root) {
    FlatBvh f;
    const BoxSlack slack(bd.bin[root].box);
    std::vector<rrt::GNode4> out;
    struct Item { int32_t bin; int32_t slot; uint32_t depth; };
    std::vector<Item> stack;
    out.push_back(rrt::GNode4{});
    stack.push_back(Item{root, 0, 0});
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        f.max_depth = std::max(f.max_depth, it.depth + 1);
        std::vector<int32_t> kids;
        const Builder::BNode &b = bd.bin[it.bin];
        if (b.leaf) kids.push_back(it.bin);
        else { kids.push_back(b.left); kids.push_back(b.right); }
        while (kids.size() < 4) {
            int best = -1;
            double best_area = -1.0;
            for (size_t i = 0; i < kids.size(); ++i) {
                const Builder::BNode &k = bd.bin[kids[i]];
                if (k.leaf) continue;
                const double area = surface_area(k.box);
                if (area > best_area) { best_area = area; best = (int)i; }
            }
            if (best < 0) break;
            const Builder::BNode &k = bd.bin[kids[best]];
            kids[best] = k.left;
            kids.insert(kids.begin() + best + 1, k.right);
        }
        float lo[4][3], hi[4][3];
        int32_t child[4], count[4];
        for (int c = 0; c < 4; ++c) {
            if (c >= (int)kids.size()) {
                put_box(lo[c], hi[c], never_hit_box(), nullptr);
                child[c] = 0;
                count[c] = 0;
                continue;
            }
            const Builder::BNode &k = bd.bin[kids[c]];
            if (k.leaf && k.count == 0) {  // empty scene: nothing to enter
                put_box(lo[c], hi[c], never_hit_box(), nullptr);
                child[c] = 0;
                count[c] = 0;
                continue;
            }
            put_box(lo[c], hi[c], k.box, &slack);
            if (k.leaf) {
                child[c] = k.first;
                count[c] = k.count;
                f.n_leaves++;
                f.max_leaf = std::max<uint32_t>(f.max_leaf, (uint32_t)k.count);
            } else {
                child[c] = (int32_t)out.size();
                count[c] = 0;
                out.push_back(rrt::GNode4{});
                stack.push_back(Item{kids[c], child[c], it.depth + 1});
            }
        }
        rrt::GNode4 &n = out[it.slot];
        n.lox = make_float4(lo[0][0], lo[1][0], lo[2][0], lo[3][0]);
        n.hix = make_float4(hi[0][0], hi[1][0], hi[2][0], hi[3][0]);
        n.loy = make_float4(lo[0][1], lo[1][1], lo[2][1], lo[3][1]);
        n.hiy = make_float4(hi[0][1], hi[1][1], hi[2][1], hi[3][1]);
        n.loz = make_float4(lo[0][2], lo[1][2], lo[2][2], lo[3][2]);
        n.hiz = make_float4(hi[0][2], hi[1][2], hi[2][2], hi[3][2]);
        n.child = make_int4(child[0], child[1], child[2], child[3]);
        n.count = make_int4(count[0], count[1], count[2], count[3]);
    }
    f.n_nodes = (uint32_t)out.size();
    f.stack_need = 3 * f.max_depth + 1;  // <= 3 pushes per level
    f.width = 4;
    f.stride = (uint32_t)sizeof(rrt::GNode4);
    f.bytes.resize(out.size() * sizeof(rrt::GNode4));
    std::memcpy(f.bytes.data(), out.data(), f.bytes.size());
    return f;
}


// The BVH's shape by kernel and node placement (scene_bvh). A scene staged in LDS is built with
// leaves of up to max_leaf (3) primitives at the SAH node price (Builder::node_cost, in sphere
// tests) of the kernel: 2 for the f32 kernel (a node visit ~ two sphere tests there), 1.5 for the
// f64 kernel, which tests boxes in f32 and spheres in f64 (C2 f64 +3.2 % same-box against 2; lower
// prices grow the tree past its block's 64 KB; profiles/r4l_f64_sah_sweep.log, r4m_f64_sah_sweep.log).
// A scene read from L2 — 32-B f16 nodes, primitive records gathered per lane — is split down to
// single-primitive leaves (the price is moot there): a node visit is two 16-B loads, a primitive
// test at least as many plus its arithmetic, and book-2 primitives cost more than a sphere test.
// Same-box against the price-2, 3-primitive tree: final_scene 9.86 -> 11.0 Grays/s, bouncing
// spheres +3.1 %, C5 +0.7 %, C5 f64 +3.7 % (profiles/r4n_*, r4o_leaf_sweep.log).
// RRT_SAH_CT (every build), RRT_F64_SAH_CT_LDS, RRT_MAX_LEAF_GLOBAL: experiments.
constexpr double kNodeCost = 2.0;
double env_or(const char *name, double v) {
    const char *e = std::getenv(name);
    return e ? std::atof(e) : v;
}
double f64_node_cost_lds() { return env_or("RRT_F64_SAH_CT_LDS", 1.5); }
uint32_t max_leaf_global() { return (uint32_t)std::max(1.0, env_or("RRT_MAX_LEAF_GLOBAL", 1)); }

// A dielectric's scatter (material.rs:83-102) divides twice per hit in f32: ri = 1 / eta on a
// front face, and Schlick's r0 = (1 - ri) / (1 + ri) squared (material.rs:75-80). Both depend on
// the material and the face only, so the host forms them once, in the same correctly rounded f32
// operations in the same order (no contraction: volatile stores round each step), into the
// dielectric's unused albedo slots: a = (1 / eta, r0(1 / eta), r0(eta), fuzz). The f64 kernel
// ignores them. RRT_DIEL_HOST=0: the kernel divides (A/B).
#ifndef RRT_DIEL_HOST
#define RRT_DIEL_HOST 1
#endif
void dielectric_consts(float eta, float &inv_eta, float &r0_front, float &r0_back) {
    auto r0sq = [](float ri) {
        volatile float num = 1.0f - ri, den = 1.0f + ri;
        volatile float q = num / den;
        volatile float q2 = q * q;
        return (float)q2;
    };
    volatile float inv = 1.0f / eta;
    inv_eta = inv;
    r0_front = r0sq(inv_eta);
    r0_back = r0sq(eta);
}

// Russian roulette's 1 / pr (camera.rs:189-200) for an attenuation that is a material constant
// (a plain Lambertian's or a metal's albedo): pr = max component clamped to [0.05, 0.95], then the
// f32 quotient the kernel would form. Only the f32 book-1 kernel reads it (b.y); the f64 kernel and
// book-2 materials keep b.y's own meaning.
#ifndef RRT_PR_HOST
#define RRT_PR_HOST 1
#endif
// An albedo as the f64 kernel's attenuation history may hold it: any NaN becomes the quiet NaN, so
// no albedo carries the signalling-NaN patterns that tag texel bytes there (its value is NaN either
// way: BOOKS propagates NaN whatever its payload).
float canonical_albedo(float a) { return a == a ? a : std::numeric_limits<float>::quiet_NaN(); }

float rr_inv_pr(float ax, float ay, float az) {
    float pr = ax;
    if (ay > pr) pr = ay;
    if (az > pr) pr = az;
    if (pr < 0.05f) pr = 0.05f;
    if (pr > 0.95f) pr = 0.95f;
    volatile float q = 1.0f / pr;
    return q;
}

// The same constants in f64 for the f64 kernel (material.rs:88-99 in the reference's f64).
void dielectric_consts64(double eta, double &inv_eta, double &r0_front, double &r0_back) {
    auto r0sq = [](double ri) {
        volatile double num = 1.0 - ri, den = 1.0 + ri;
        volatile double q = num / den;
        volatile double q2 = q * q;
        return (double)q2;
    };
    volatile double inv = 1.0 / eta;
    inv_eta = inv;
    r0_front = r0sq(inv_eta);
    r0_back = r0sq(eta);
}

// Default BVH shape of scene creation (env knobs are for experiments).
void bvh_defaults(uint32_t &width, uint32_t &max_leaf) {
    max_leaf = 3;
    if (const char *e = std::getenv("RRT_MAX_LEAF")) max_leaf = (uint32_t)std::min(15, std::max(1, std::atoi(e)));
    width = 2;
    if (const char *e = std::getenv("RRT_BVH_WIDTH")) width = std::atoi(e) == 4 ? 4 : 2;
    if (width == 2) max_leaf = std::min(max_leaf, rrt::kMaxLeafPrims);
}

// Quad::set_bounding_box (quad.rs:43-47): the box of the four corners, padded.
static Aabb quad_box(const RrtQuad &qd) {
    Aabb b;
    for (int a = 0; a < 3; ++a) {
        const double q = qd.q[a], u = qd.u[a], v = qd.v[a];
        const double c[4] = {q, q + u + v, q + u, q + v};
        b.ax[a] = Interval{std::min(std::min(c[0], c[1]), std::min(c[2], c[3])),
                           std::max(std::max(c[0], c[1]), std::max(c[2], c[3]))};
    }
    return pad(b);
}

// Book-2 extension arrays with null-safe counts.
struct ExtView {
    const float *motion = nullptr;
    const RrtQuad *quads = nullptr;
    uint32_t n_quads = 0;
    const RrtMedium *media = nullptr;
    uint32_t n_media = 0;
    const RrtQuad *bquads = nullptr;
    uint32_t n_bquads = 0;
    const RrtLight *lights = nullptr;
    uint32_t n_lights = 0;
    explicit ExtView(const RrtSceneExt *e) {
        if (!e) return;
        motion = e->sphere_motion;
        if (e->quads) quads = e->quads, n_quads = e->n_quads;
        if (e->media) media = e->media, n_media = e->n_media;
        if (e->boundary_quads) bquads = e->boundary_quads, n_bquads = e->n_boundary_quads;
        if (e->lights) lights = e->lights, n_lights = e->n_lights;
    }
};

// Sphere boxes (sphere.rs:16-21, aabb.rs:29-34: r = max(radius, 0), padded; a moving sphere's
// box spans both ends, the_next_week/sphere.rs:31-33), quad boxes, medium boxes (the boundary's:
// constant_medium.rs bounding_box), SAH build, flatten. Primitives: spheres, then quads
// (n_spheres + j), then media (n_spheres + n_quads + m). order[i] = original index of the i-th
// primitive in leaf order. The medium ranges are validated by the caller.
// Whether nodes + primitive records (+ motion for book-2 kernels) are staged in LDS per block
// (RRT_SCENE_IN_LDS=0 forces global memory).
bool scene_lds_forced_off() {
    const char *e = std::getenv("RRT_SCENE_IN_LDS");
    return e && std::atoi(e) == 0;
}
bool scene_lds_fit(size_t node_bytes, size_t n_prims, bool book2) {
    if (scene_lds_forced_off()) return false;
    return node_bytes + n_prims * (rrt::kPrimBytes + (book2 ? rrt::kMotionBytes : 0)) <= rrt::kLdsSceneBudget;
}

// The unbounded media (FlatBvh::n_unbounded), in medium order, at most kMaxUnbounded: a
// sphere-bounded medium whose box [c - r, c + r] holds every other primitive's extent — sphere
// boxes (both ends of a motion), quad corners q, q + u, q + v, (q + u) + v, the other media's
// boundaries — in f64 from the f32 inputs. Only a scheduling choice: a medium's hit does not
// depend on when the query tests it (its free flight is clipped to the closest hit so far, and
// the per-(path, segment, medium) draw is fixed), so testing it after the walk returns the same
// closest hit. The oracle's f32 modes restate the rule (oracle/rrt_oracle.cpp unbounded_media).
std::vector<uint32_t> unbounded_media(const RrtSphere *spheres, uint32_t n_spheres, const ExtView &ex) {
    std::vector<uint32_t> out;
    for (uint32_t m = 0; m < ex.n_media && out.size() < rrt::kMaxUnbounded; ++m) {
        const RrtMedium &md = ex.media[m];
        if (md.boundary_kind != RRT_BOUNDARY_SPHERE) continue;
        const double r = std::max((double)md.sphere[3], 0.0);
        double lo[3], hi[3];
        for (int a = 0; a < 3; ++a) lo[a] = (double)md.sphere[a] - r, hi[a] = (double)md.sphere[a] + r;
        bool ok = true;
        auto pt = [&](double x, double y, double z, double e) {
            const double v[3] = {x, y, z};
            for (int a = 0; a < 3; ++a) ok = ok && lo[a] <= v[a] - e && v[a] + e <= hi[a];
        };
        auto quad = [&](const RrtQuad &q) {
            pt(q.q[0], q.q[1], q.q[2], 0.0);
            pt((double)q.q[0] + q.u[0], (double)q.q[1] + q.u[1], (double)q.q[2] + q.u[2], 0.0);
            pt((double)q.q[0] + q.v[0], (double)q.q[1] + q.v[1], (double)q.q[2] + q.v[2], 0.0);
            pt(((double)q.q[0] + q.u[0]) + q.v[0], ((double)q.q[1] + q.u[1]) + q.v[1], ((double)q.q[2] + q.u[2]) + q.v[2], 0.0);
        };
        for (uint32_t i = 0; i < n_spheres && ok; ++i) {
            const float *c = spheres[i].center_radius;
            const double ri = std::max((double)c[3], 0.0);
            pt(c[0], c[1], c[2], ri);
            if (ex.motion) {
                const float *mv = ex.motion + 4 * (size_t)i;
                pt((double)(c[0] + mv[0]), (double)(c[1] + mv[1]), (double)(c[2] + mv[2]), ri);
            }
        }
        for (uint32_t j = 0; j < ex.n_quads && ok; ++j) quad(ex.quads[j]);
        for (uint32_t k = 0; k < ex.n_media && ok; ++k) {
            if (k == m) continue;
            const RrtMedium &o = ex.media[k];
            if (o.boundary_kind == RRT_BOUNDARY_SPHERE) pt(o.sphere[0], o.sphere[1], o.sphere[2], std::max((double)o.sphere[3], 0.0));
            else for (uint32_t q = 0; q < o.count && ok; ++q) quad(ex.bquads[o.first + q]);
        }
        if (ok) out.push_back(m);
    }
    return out;
}

// BVH2 node layout: the sign-ordered 80-B nodes when `lds_fit(the tree in those nodes)` says the
// scene will be staged in LDS, else the 32-B f16 global-memory nodes. node_cost: the SAH's node
// visit price in sphere tests (Builder::node_cost).
FlatBvh build_bvh(const RrtSphere *spheres, uint32_t n_spheres, const ExtView &ex, uint32_t width,
                  uint32_t max_leaf, double node_cost, std::vector<uint32_t> &order,
                  const std::function<bool(const FlatBvh &)> &lds_fit) {
    const float *motion = ex.motion;
    const uint32_t n_quads = ex.n_quads;
    std::vector<Aabb> boxes(n_spheres + (size_t)n_quads + ex.n_media);
    for (uint32_t i = 0; i < n_spheres; ++i) {
        const double r = std::max((double)spheres[i].center_radius[3], 0.0);
        Aabb b;
        for (int a = 0; a < 3; ++a) {
            const double c = spheres[i].center_radius[a];
            b.ax[a] = Interval{c - r, c + r};
            if (motion) {  // center2 = center1 + motion (f32 sum, as the kernel's t = 1 end)
                const double c2 = (double)(spheres[i].center_radius[a] + motion[4 * (size_t)i + a]);
                b.ax[a] = iv_union(b.ax[a], Interval{c2 - r, c2 + r});
            }
        }
        boxes[i] = pad(b);
    }
    for (uint32_t j = 0; j < n_quads; ++j) boxes[n_spheres + j] = quad_box(ex.quads[j]);
    for (uint32_t m = 0; m < ex.n_media; ++m) {
        const RrtMedium &md = ex.media[m];
        Aabb b = aabb_empty();
        if (md.boundary_kind == RRT_BOUNDARY_SPHERE) {
            const double r = std::max((double)md.sphere[3], 0.0);
            for (int a = 0; a < 3; ++a) b.ax[a] = Interval{md.sphere[a] - r, md.sphere[a] + r};
            b = pad(b);
        } else {
            for (uint32_t k = 0; k < md.count; ++k) b = aabb_union(b, quad_box(ex.bquads[md.first + k]));
        }
        boxes[n_spheres + n_quads + m] = b;
    }
    const uint32_t n_prims = n_spheres + n_quads + ex.n_media;
    const std::vector<uint32_t> unb = unbounded_media(spheres, n_spheres, ex);
    Builder bld(boxes, max_leaf);
    for (uint32_t m : unb) bld.objs.erase(std::find(bld.objs.begin(), bld.objs.end(), n_spheres + n_quads + m));
    const uint32_t n_tree = (uint32_t)bld.objs.size();
    if (const char *e = std::getenv("RRT_BVH_SPLIT")) bld.sweep = std::strcmp(e, "binned") != 0;
    bld.node_cost = node_cost;
    if (const char *e = std::getenv("RRT_SAH_CT")) bld.node_cost = std::atof(e);
    FlatBvh fb;
    if (n_tree == 0) {  // root with never-hit children
        Builder::BNode empty;
        empty.box = never_hit_box();
        empty.leaf = true;
        bld.bin.push_back(empty);
    }
    (void)n_prims;
    const int32_t root = n_tree == 0 ? 0 : bld.build(0, n_tree);
    if (width == 4) {
        fb = flatten4(bld, root);
    } else {
        fb = flatten2<rrt::GNode>(bld, root);
        if (!lds_fit(fb)) fb = flatten2<rrt::GNodeH>(bld, root);
    }
    order = bld.objs;
    for (uint32_t m : unb) order.push_back(n_spheres + n_quads + m);
    fb.n_unbounded = (uint32_t)unb.size();
    return fb;
}

// The scene's BVH2 (the shapes above): first the LDS shape, kept when the kernel's LDS fit takes
// its sign-ordered nodes; else the global-memory shape in f16 nodes, and for the f64 kernel the LDS
// shape in f16 nodes if the global one needs more nodes than its 16-bit links and stack address.
// Width 4 (an experiment) keeps the f32 LDS shape.
FlatBvh scene_bvh(const RrtSphere *spheres, uint32_t n_spheres, const ExtView &ex, uint32_t width,
                  uint32_t max_leaf, bool book2, bool f64, std::vector<uint32_t> &order) {
    const size_t n_prims_all = (size_t)n_spheres + ex.n_quads + ex.n_media;
    std::function<bool(const FlatBvh &)> fit = [&](const FlatBvh &t) {
        return scene_lds_fit(t.bytes.size(), n_prims_all, book2);
    };
    if (f64)
        fit = [&](const FlatBvh &t) {
            return !scene_lds_forced_off() &&
                   rrt::f64_lds_min_bytes(t.n_nodes, (uint32_t)n_prims_all, t.stack_need) <= 64u * 1024u;
        };
    if (width != 2) return build_bvh(spheres, n_spheres, ex, width, max_leaf, kNodeCost, order, fit);
    FlatBvh fb = build_bvh(spheres, n_spheres, ex, width, max_leaf, f64 ? f64_node_cost_lds() : kNodeCost, order, fit);
    if (fb.stride == (uint32_t)sizeof(rrt::GNode)) return fb;
    fb = build_bvh(spheres, n_spheres, ex, width, std::min(max_leaf, max_leaf_global()), kNodeCost, order, fit);
    // the caller's leaf size when single-primitive leaves need more than the f64 kernel's 16-bit
    // links, or a deeper stack than the kernels hold (coincident spheres: the SAH sweep splits ties
    // 1 | n - 1, so a cluster of n turns into a chain n deep)
    if ((f64 && fb.n_nodes > 65535u) || fb.stack_need > (uint32_t)rrt::kMaxStackDepth)
        fb = build_bvh(spheres, n_spheres, ex, width, max_leaf, kNodeCost, order, fit);
    return fb;
}

}  // namespace

// ------------------------------------------------------------------------------------
struct RrtScene {
    int device = 0;
    uint8_t *d_nodes = nullptr;
    float4 *d_prim_cr = nullptr;
    rrt::GMaterial *d_prim_mtl = nullptr;
    double *d_prim_inv_r64 = nullptr;  // f64 scenes: 1 / r per leaf-order sphere
    double4 *d_prim_diel64 = nullptr;  // f64 scenes: dielectric constants per leaf-order sphere
    float4 *d_prim_motion = nullptr;
    rrt::GPerlin *d_perlin = nullptr;
    rrt::GQuad *d_quads = nullptr;
    rrt::GMedium *d_media = nullptr;
    rrt::GLight *d_lights = nullptr;
    uint8_t *d_tex_pool = nullptr;
    rrt::GTexture *d_texs = nullptr;
    unsigned long long *d_counters = nullptr;       // 5 x u64, render launches
    unsigned long long *d_work_counters = nullptr;  // 5 x u64, instrumented launches
    uint32_t *d_unit_counter = nullptr;             // persistent-queue head
    rrt::F3 *d_partial = nullptr;                   // chunk partial sums (RGB)
    size_t partial_cap = 0;                         // F3 elements
    bool f64 = false;                               // RRT_FLAG_F64: the books-arithmetic kernel
    rrt::D4 *d_partial64 = nullptr;                 // its chunk partial sums
    size_t partial64_cap = 0;                       // D4 elements
    rrt::D4 *d_accum64 = nullptr;                   // its f64 sums behind the float entry points
    double *d_seq64 = nullptr;                      // f64: tail-sample radiances of a pass
    size_t seq64_cap = 0;                           // doubles
    float *d_hist = nullptr;                        // f64: the lanes' attenuation histories
    size_t hist_cap = 0;                            // bytes
    size_t accum64_cap = 0;                         // D4 elements
    uint32_t last_groups = 0, last_passes = 0;      // the last launch: 64-unit groups per pass, passes
    rrt::KParams base{};
    RrtBvhInfo info{};
};

namespace {

void free_scene(RrtScene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipFree(s->d_nodes);
    (void)hipFree(s->d_prim_cr);
    (void)hipFree(s->d_prim_mtl);
    (void)hipFree(s->d_prim_inv_r64);
    (void)hipFree(s->d_prim_diel64);
    (void)hipFree(s->d_prim_motion);
    (void)hipFree(s->d_perlin);
    (void)hipFree(s->d_quads);
    (void)hipFree(s->d_media);
    (void)hipFree(s->d_lights);
    (void)hipFree(s->d_tex_pool);
    (void)hipFree(s->d_texs);
    (void)hipFree(s->d_counters);
    (void)hipFree(s->d_work_counters);
    (void)hipFree(s->d_unit_counter);
    (void)hipFree(s->d_partial);
    (void)hipFree(s->d_partial64);
    (void)hipFree(s->d_accum64);
    (void)hipFree(s->d_seq64);
    (void)hipFree(s->d_hist);
    delete s;
}

template <class T>
int upload(T **dst, const T *src, size_t n, const char *what) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    HIP_TRY(hipMalloc((void **)dst, bytes), std::string("hipMalloc ") + what);
    if (n) HIP_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice), std::string("copy ") + what);
    return RRT_OK;
}

// Serpentine band dealing (include/rrt_hip.h RrtTile): the tile's j-th band is image band
// j * n_ranks + band_slot(t, j). Round-robin (slot = rank in every period) gave rank n-1 the
// lowest band of every period, so on C3 its tile was the most expensive: 1.96 % over the mean at 8
// ranks (tools/c3_rank_balance.py); alternating the order per period cancels that trend.
uint32_t band_slot(const RrtTile &t, uint32_t j) { return (j & 1u) ? t.n_ranks - 1u - t.rank : t.rank; }

uint32_t tile_rows_of(uint32_t height, const RrtTile &t) {
    uint32_t rows = 0;
    const uint32_t bands = (height + t.band_rows - 1) / t.band_rows;
    for (uint32_t j = 0;; ++j) {
        const uint32_t b = j * t.n_ranks + band_slot(t, j);
        if (j * t.n_ranks >= bands) break;
        if (b < bands) rows += std::min(t.band_rows, height - b * t.band_rows);
    }
    return rows;
}

int check_tile_shape(const RrtTile *t) {
    if (!t) return fail(RRT_E_INVALID, "null tile");
    if (t->band_rows == 0 || t->n_ranks == 0 || t->rank >= t->n_ranks)
        return fail(RRT_E_INVALID, "tile: band_rows and n_ranks must be > 0 and rank < n_ranks");
    if (t->sample_end < t->sample_begin) return fail(RRT_E_INVALID, "tile: sample_end < sample_begin");
    return RRT_OK;
}

int check_tile(const RrtScene *s, const RrtTile *t) {
    if (!s) return fail(RRT_E_INVALID, "null scene");
    if (int rc = check_tile_shape(t)) return rc;
    const uint32_t sq = s->base.sqrt_spp;
    if (sq && (uint64_t)t->sample_end > (uint64_t)sq * sq)  // book 3: s = s_j * sqrt_spp + s_i
        return fail(RRT_E_INVALID, "RRT_FLAG_BOOK3: sample_end exceeds sqrt_spp^2 = " + std::to_string(sq * sq));
    return RRT_OK;
}

// Free device memory (0 when the query fails): the f64 path sizes its buffers within it.
size_t device_free_bytes(int device) {
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 0;
    return free_b;
}

// Bytes of chunk partials one render may hold (RRT_PARTIAL_MB, default 2048 MiB): C2 (15 x
// 33 MB) renders in one pass, a whole C3 frame on one GPU (39 x 133 MB) in three.
size_t partial_budget() {
    size_t mb = 2048;
    if (const char *e = std::getenv("RRT_PARTIAL_MB")) mb = (size_t)std::max(1, std::atoi(e));
    return mb << 20;
}

// The f64 path's tail-sample radiances (24 B per nonzero sample + a 4-B mask per tail unit and
// pixel): 8 GiB, at most half the device's free memory, unless RRT_PARTIAL_MB says otherwise — C2's
// 128 tail samples of 2.07 M pixels (6.4 GB) in one pass of the 288-GB HBM; a smaller device runs
// more sample passes instead of failing its allocation.
size_t seq_budget(int device) {
    if (std::getenv("RRT_PARTIAL_MB")) return partial_budget();
    return std::min((size_t)8192 << 20, std::max(device_free_bytes(device) / 2, (size_t)64 << 20));
}
#ifndef RRT_F64_SEQ
#define RRT_F64_SEQ 1
#endif
#ifndef RRT_F64_TAIL_DIV
#define RRT_F64_TAIL_DIV 4
#endif
// frames of more than 512 samples (C4, C3): T = S/2, prefix units of S/2 samples. Same-box against
// S/4: C4 +4 %; the same rule at 512 samples and below: C2 -4.5 %, C5 -5 % (r5_f64_ab_batch6.log)
#ifndef RRT_F64_TAIL_DIV_HI
#define RRT_F64_TAIL_DIV_HI 2
#endif
#ifndef RRT_F64_TS_DIV  // the f64 tail units: K/8 samples
#define RRT_F64_TS_DIV 8
#endif

int fill_params(RrtScene *s, const RrtTile *t, float *d_accum, rrt::KParams &p) {
    p = s->base;
    p.accum = reinterpret_cast<float4 *>(d_accum);
    p.tile_rows = tile_rows_of(p.height, *t);
    p.band_rows = t->band_rows;
    p.rank = t->rank;
    p.n_ranks = t->n_ranks;
    p.sample_begin = t->sample_begin;
    p.sample_end = t->sample_end;
    p.tiles_x = (p.width + rrt::kTileW - 1u) / rrt::kTileW;
    p.n_work_tiles = p.tiles_x * ((p.tile_rows + rrt::kTileH - 1u) / rrt::kTileH);
    const uint32_t S = t->sample_end - t->sample_begin;
    // the frame's chunk (rrt_accum_chunk = K0): halved while S <= 2K, down to K0/4 — big chunks pay
    // at high spp (per-unit cost), small ones at low spp (drain granularity). K0 = 256: S > 512 ->
    // 256 (C4, C3), 256 < S <= 512 -> 128 (C2), S <= 256 -> 64 (C5)
    const uint32_t k0 = p.chunk;
    while (p.chunk > std::max(1u, k0 / 4u) && S <= 2u * p.chunk) p.chunk /= 2u;
#ifdef RRT_CHUNK_FORCE  // A/B builds only (tools/build_variants.sh): a fixed chunk outside the ABI's rule
    p.chunk = std::max(1u, (uint32_t)RRT_CHUNK_FORCE);
#endif
// tail chunks of K/4 (ABI v10; K/8 before): a quarter of C2's chunk partials fewer (7 instead of 11
// per pixel, ~100 MB less HBM written and read per launch), same-box C2 +0.3 %, C4 +0.6 %, C5 ±0.2 %.
// Frames of at most K0/4 samples, which are all tail (no big chunk), keep K/8 (ABI v11): their units
// are few per lane, so the queue's drain is what the small chunks buy — same-box final_scene
// (64 spp) +6.4 % over K/4 (profiles/r5_ab_tail_div.log)
#ifndef RRT_TAIL_DIV
#define RRT_TAIL_DIV 4
#endif
#ifndef RRT_TAIL_DIV_LO
#define RRT_TAIL_DIV_LO 8
#endif
    p.chunk_small = std::max(1u, p.chunk / (S <= k0 / 4u ? RRT_TAIL_DIV_LO : RRT_TAIL_DIV));
    p.n_big = S > p.chunk ? (S - 1u) / p.chunk : 0u;
    const uint32_t tail = S - p.n_big * p.chunk;
    p.n_chunks = S ? p.n_big + (tail + p.chunk_small - 1u) / p.chunk_small : 0u;
    p.seq = 0u;
    if (s->f64 && RRT_F64_SEQ && S) {
        // The f64 books path sums each pixel's samples in camera.rs:72-76's order: one prefix chunk
        // of S - T samples (summed in the lane from 0), then T tail samples in chunks of K/8 whose
        // radiances are kept one by one and folded in after the pass. T = S/4 in whole tail chunks
        // (C2: 128 samples in 8 chunks of 16): it balances the queue's drain as well as the chunked
        // schedule did (same-box C2 18.75 vs 18.73 Grays/s); T = S/8 left the drain uncovered (-5 %).
        // T = S/2 above 512 samples.
        const uint32_t ts = std::min(std::max(1u, p.chunk / RRT_F64_TS_DIV), 32u);  // a tail unit's mask is 32 bits
        const uint32_t tdiv = S > 512u ? RRT_F64_TAIL_DIV_HI : RRT_F64_TAIL_DIV;
        const uint32_t t_samples = S >= 2u * ts ? (S / tdiv) / ts * ts : 0u;
        p.seq = 1u;
        p.n_big = 1u;
        p.chunk = S - t_samples;
        p.chunk_small = ts;
        p.n_chunks = 1u + t_samples / ts;
    }
    const uint64_t units = (uint64_t)p.n_work_tiles * p.n_chunks * 64u;
    if (units > 0xFFFFFFFFull) return fail(RRT_E_INVALID, "tile too large: more than 2^32 work units");
    p.n_units = (uint32_t)units;
    p.n_big_units = p.n_work_tiles * p.n_big * 64u;
    p.fd_tiles_x = rrt::make_fastdiv(p.tiles_x);
    p.fd_band_rows = rrt::make_fastdiv(p.band_rows);
    p.fd_n_ranks = rrt::make_fastdiv(p.n_ranks);
    p.fd_chunk = rrt::make_fastdiv(p.chunk);
    p.fd_chunk_small = rrt::make_fastdiv(p.chunk_small);
    p.fd_sqrt_spp = rrt::make_fastdiv(p.sqrt_spp);
    p.fd_pass_big = rrt::make_fastdiv(p.n_big);
    p.fd_pass_tail = rrt::make_fastdiv(p.n_chunks - p.n_big);
    p.unit_counter = s->d_unit_counter;
    p.pass_chunks = p.n_chunks;
    if (p.seq && p.n_chunks > 1) {  // per-sample tail radiances [pass tail sample][pixel], within the budget
        const size_t n_px = std::max<size_t>((size_t)p.tile_rows * p.width, 1);
        const size_t per_chunk = n_px * p.chunk_small * 3u * sizeof(double) + n_px * sizeof(uint32_t);
        const uint32_t n_tail = p.n_chunks - 1u;
        p.pass_chunks = (uint32_t)std::min<size_t>(n_tail, std::max<size_t>(1, seq_budget(s->device) / per_chunk));
        const size_t need = (per_chunk * p.pass_chunks + sizeof(double) - 1) / sizeof(double);
        if (need > s->seq64_cap) {
            HIP_TRY(hipSetDevice(s->device), "hipSetDevice");
            (void)hipFree(s->d_seq64);
            s->d_seq64 = nullptr;
            s->seq64_cap = 0;
            HIP_TRY(hipMalloc((void **)&s->d_seq64, need * sizeof(double)), "hipMalloc tail sample radiances");
            s->seq64_cap = need;
        }
    } else if (p.n_chunks > 1) {  // partial sums [pass chunk][pixel], within the partial budget; grow on demand
        const size_t n_px = std::max<size_t>((size_t)p.tile_rows * p.width, 1);
        const size_t elem = s->f64 ? sizeof(rrt::D4) : sizeof(rrt::F3);
        p.pass_chunks = (uint32_t)std::min<size_t>(p.n_chunks, std::max<size_t>(1, partial_budget() / (n_px * elem)));
        const size_t need = n_px * p.pass_chunks;
        size_t &cap = s->f64 ? s->partial64_cap : s->partial_cap;
        void **buf = s->f64 ? (void **)&s->d_partial64 : (void **)&s->d_partial;
        if (need > cap) {
            HIP_TRY(hipSetDevice(s->device), "hipSetDevice");
            (void)hipFree(*buf);
            *buf = nullptr;
            cap = 0;
            HIP_TRY(hipMalloc(buf, need * elem), "hipMalloc chunk partials");
            cap = need;
        }
    }
    p.partial = s->d_partial;
    p.partial64 = s->d_partial64;
    p.seq64 = s->d_seq64;
    p.seqmask = nullptr;
    if (p.seq && p.n_chunks > 1) {  // the masks follow the pass's packed radiances
        const size_t n_px = std::max<size_t>((size_t)p.tile_rows * p.width, 1);
        p.seqmask = reinterpret_cast<uint32_t *>(s->d_seq64 + (size_t)p.pass_chunks * n_px * p.chunk_small * 3u);
    }
    p.accum64 = nullptr;
    if (s->f64) {  // the attenuation history: max_depth records of 12 B per lane slot
        const uint64_t per_lane = (uint64_t)std::max(1u, p.max_depth) * 12u;
#ifndef RRT_F64_HIST_LANES_PER_CU
#define RRT_F64_HIST_LANES_PER_CU 1024  // 4 waves per SIMD x 4 SIMDs x 64 (the f64 kernel's bound)
#endif
        // Every lane the persistent grid holds gets a slot. Within half the device's free memory
        // (C2: 315 MB; depth 5000: 15.7 GB), so a deep max_depth costs memory, not occupancy; only
        // beyond that is the grid cut to the lanes that fit, and the render says so on stderr.
        const uint64_t full = (uint64_t)p.n_cus * RRT_F64_HIST_LANES_PER_CU;
        uint64_t lanes = full;
        if (lanes * per_lane > s->hist_cap) {
            const uint64_t room = std::max<uint64_t>(device_free_bytes(s->device) + s->hist_cap, 1ull << 30) / 2u;
            lanes = std::min<uint64_t>(lanes, room / per_lane / 512u * 512u);
        } else {
            lanes = std::min<uint64_t>(lanes, s->hist_cap / per_lane);
        }
        if (lanes < 8u * 512u) return fail(RRT_E_INVALID, "RRT_FLAG_F64: max_depth too large for the attenuation history");
        if (lanes < full)
            std::fprintf(stderr, "rrt: RRT_FLAG_F64 max_depth %u: attenuation history for %llu of %llu lanes; the grid is reduced to fit\n",
                         p.max_depth, (unsigned long long)lanes, (unsigned long long)full);
        const size_t need = (size_t)(lanes * per_lane);
        if (need > s->hist_cap) {
            HIP_TRY(hipSetDevice(s->device), "hipSetDevice");
            (void)hipFree(s->d_hist);
            s->d_hist = nullptr;
            s->hist_cap = 0;
            HIP_TRY(hipMalloc((void **)&s->d_hist, need), "hipMalloc attenuation history");
            s->hist_cap = need;
        }
        p.hist = s->d_hist;
        p.hist_lanes = (uint32_t)std::min<uint64_t>(s->hist_cap / per_lane, 0xFFFFFFFFull);
    }
    return RRT_OK;
}

// The largest big chunk K0 (tail chunks K/4, K/8 for frames of at most K0/4 samples; the frame's K: rrt_accum_chunk's rule, halved while
// S <= 2K down to K0/4). 128 in round 2 (with 8 work queues the per-unit cost matters more than the
// drain: C2 +1.2 %, C4 +10 %, C5 -0.5 % against 64); 256 since round 4 for frames over 512 samples:
// C4 +2.4 %, C3 +0.8 % same-box, C2 and C5 keep 128 and 64 (K = 256 at C2's 512 spp: -0.3 %).
uint32_t accum_chunk() {
    uint32_t c = 256;
    if (const char *e = std::getenv("RRT_CHUNK")) c = (uint32_t)std::max(1, std::atoi(e));
    return c;
}

}  // namespace

extern "C" {

const char *rrt_hip_last_error(void) { return g_err.c_str(); }
uint32_t rrt_accum_chunk(void) { return accum_chunk(); }
uint32_t rrt_hip_abi_version(void) { return RRT_ABI_VERSION; }

int32_t rrt_device_count(int32_t *count) {
    if (!count) return fail(RRT_E_INVALID, "null count");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RRT_OK;
}

}  // extern "C"

static int32_t scene_create(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                            uint32_t n_textures, const RrtSceneExt *ext, uint32_t flags, int32_t device,
                            RrtScene **out) {
    if (!cam || !out) return fail(RRT_E_INVALID, "null camera or out pointer");
    ExtView ex(ext);
    const float *motion = ex.motion;
    const uint32_t n_perlin = ext && ext->perlin ? ext->n_perlin : 0u;
    const RrtQuad *quads = ex.quads;
    const uint32_t n_quads = ex.n_quads;
    for (uint32_t j = 0; j < n_quads; ++j) {
        if (quads[j].material_index >= n_materials)
            return fail(RRT_E_INVALID, "quad " + std::to_string(j) + " material_index out of range");
        if (materials[quads[j].material_index].kind == RRT_MAT_TEXTURED_LAMBERTIAN)
            return fail(RRT_E_INVALID, "quad " + std::to_string(j) + ": image textures on quads are not supported");
    }
    const uint32_t n_media = ex.n_media;
    for (uint32_t m = 0; m < n_media; ++m) {
        const RrtMedium &md = ex.media[m];
        const std::string what = "medium " + std::to_string(m);
        if (md.material_index >= n_materials || materials[md.material_index].kind != RRT_MAT_ISOTROPIC)
            return fail(RRT_E_INVALID, what + ": material_index must name an RRT_MAT_ISOTROPIC material");
        if (!(md.density > 0.0f) || !std::isfinite(md.density))
            return fail(RRT_E_INVALID, what + ": density must be positive and finite");
        if (md.boundary_kind == RRT_BOUNDARY_QUADS) {
            if (md.count == 0 || (uint64_t)md.first + md.count > ex.n_bquads)
                return fail(RRT_E_INVALID, what + ": boundary quad range out of bounds");
        } else if (md.boundary_kind != RRT_BOUNDARY_SPHERE) {
            return fail(RRT_E_INVALID, what + ": unknown boundary_kind");
        }
    }
    bool has_motion = false;
    if (motion)
        for (size_t i = 0; i < (size_t)n_spheres * 4 && !has_motion; ++i)
            has_motion = (i % 4 != 3) && motion[i] != 0.0f;
    if (has_motion && !(flags & RRT_FLAG_RAY_TIME))
        return fail(RRT_E_INVALID, "moving spheres need RRT_FLAG_RAY_TIME (rays carry the camera's time draw)");
    // Book-2 scenes (moving spheres or checker / noise materials) take the kernel variant that
    // supports them; it reads a motion row per sphere (zero for static spheres).
    const bool book3 = (flags & RRT_FLAG_BOOK3) != 0;
    uint32_t sqrt_spp = 0;
    if (book3) {
        if (!(flags & RRT_FLAG_RAY_TIME)) return fail(RRT_E_INVALID, "RRT_FLAG_BOOK3 needs RRT_FLAG_RAY_TIME");
        if (ex.n_lights == 0) return fail(RRT_E_INVALID, "RRT_FLAG_BOOK3 needs a non-empty RrtSceneExt.lights");
        const uint32_t spp = (uint32_t)std::max(cam->params_f[3], 1.0f);
        sqrt_spp = (uint32_t)std::sqrt((double)spp);
        if (sqrt_spp * sqrt_spp != spp)
            return fail(RRT_E_INVALID, "RRT_FLAG_BOOK3 samples_per_pixel must be a square (sqrt_spp^2, camera.rs:115-117)");
        for (uint32_t l = 0; l < ex.n_lights; ++l)
            if (ex.lights[l].kind > RRT_LIGHT_SPHERE)
                return fail(RRT_E_INVALID, "light " + std::to_string(l) + ": unknown kind");
    }
    bool book2 = has_motion || n_quads > 0 || n_media > 0 || book3;
    for (uint32_t i = 0; i < n_materials && materials; ++i)
        book2 = book2 || materials[i].kind == RRT_MAT_CHECKER_LAMBERTIAN || materials[i].kind == RRT_MAT_NOISE_LAMBERTIAN ||
                materials[i].kind == RRT_MAT_ISOTROPIC;
    static_assert(RRT_FLAG_F64 == rrt::kFlagF64, "RRT_FLAG_F64");
    const bool f64 = (flags & RRT_FLAG_F64) != 0;
    if (f64 && (book2 || n_perlin || ex.n_lights))
        return fail(RRT_E_INVALID, "RRT_FLAG_F64 renders book-1 scenes (material kinds 0-4, no RrtSceneExt data, "
                                   "not RRT_FLAG_BOOK3)");
    if (!has_motion) motion = nullptr;
    if (n_spheres && !spheres) return fail(RRT_E_INVALID, "null spheres");
    if (n_materials && !materials) return fail(RRT_E_INVALID, "null materials");
    if (n_textures && !textures) return fail(RRT_E_INVALID, "null textures");
    *out = nullptr;
    const float wf = cam->params_f[1], hf = cam->params_f[2];
    if (!(wf >= 1.0f) || !(hf >= 1.0f) || wf > 65536.0f || hf > 65536.0f)
        return fail(RRT_E_INVALID, "camera params_f[1..2] (width/height) out of range");
    for (uint32_t i = 0; i < n_spheres; ++i)
        if (spheres[i].material_index >= n_materials)
            return fail(RRT_E_INVALID, "sphere " + std::to_string(i) + " material_index out of range");
    for (uint32_t i = 0; i < n_materials; ++i) {
        if (materials[i].kind > RRT_MAT_ISOTROPIC)
            return fail(RRT_E_INVALID, "material " + std::to_string(i) + " has unknown kind");
        if (materials[i].kind == RRT_MAT_TEXTURED_LAMBERTIAN && materials[i]._pad[0] >= n_textures)
            return fail(RRT_E_INVALID, "material " + std::to_string(i) + " texture index out of range");
        if (materials[i].kind == RRT_MAT_NOISE_LAMBERTIAN && materials[i]._pad[0] >= n_perlin)
            return fail(RRT_E_INVALID, "material " + std::to_string(i) + " Perlin table index out of range");
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RRT_E_NODEV, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(RRT_E_INVALID, "device index out of range");

    // ---- BVH over the sphere bounding boxes ----
    uint32_t width, max_leaf;
    bvh_defaults(width, max_leaf);
    if (book2 || f64) width = 2;  // the book-2 and f64 kernels are BVH2 only
    std::vector<uint32_t> order;
    if ((uint64_t)n_spheres + n_quads + n_media >= (1u << 24) ||
        (uint64_t)n_quads + ex.n_bquads + ex.n_lights >= (1u << 24))
        return fail(RRT_E_INVALID, ">= 2^24 primitives or quads");
    if (!has_motion) ex.motion = nullptr;
    const FlatBvh fb = scene_bvh(spheres, n_spheres, ex, width, max_leaf, book2, f64, order);
    if (fb.stack_need > (uint32_t)rrt::kMaxStackDepth)
        return fail(RRT_E_INVALID, "BVH depth " + std::to_string(fb.max_depth) + " exceeds the LDS stack");
    if (f64 && fb.n_nodes > 65535u) return fail(RRT_E_INVALID, "RRT_FLAG_F64: more than 65535 BVH nodes");
    // postponed leaf tests pack (first primitive, count) as first | count << 28
    if (fb.max_leaf > (fb.width == 2 ? rrt::kMaxLeafPrims : 15u)) return fail(RRT_E_INVALID, "leaf size too large");
    if (!fb.sibling_leaves_adjacent) return fail(RRT_E_INVALID, "internal: BVH2 sibling leaves not adjacent");
    const uint32_t n_prims = n_spheres + n_quads + n_media;

    std::vector<rrt::GMaterial> mats(n_materials);
    for (uint32_t i = 0; i < n_materials; ++i) {
        const RrtMaterial &m = materials[i];
        float fuzz = m.albedo_fuzz[3];
        if (m.kind == RRT_MAT_METAL) fuzz = fuzz < 1.0f ? fuzz : 1.0f;  // material.rs:48-50
        int ref_bits;
        std::memcpy(&ref_bits, &m.ref_idx, 4);
        mats[i].a = make_float4(m.albedo_fuzz[0], m.albedo_fuzz[1], m.albedo_fuzz[2], fuzz);
        if (f64) {  // canonical_albedo: the f64 history tags texel bytes as signalling NaNs (rrt_books64.hip kTexelTag)
            mats[i].a.x = canonical_albedo(mats[i].a.x);
            mats[i].a.y = canonical_albedo(mats[i].a.y);
            mats[i].a.z = canonical_albedo(mats[i].a.z);
        }
        mats[i].b = make_int4((int)m.kind, ref_bits, (int)m._pad[0], (int)m._pad[1]);
        if ((m.kind == RRT_MAT_LAMBERTIAN || m.kind == RRT_MAT_METAL) && RRT_PR_HOST) {
            const float inv_pr = rr_inv_pr(m.albedo_fuzz[0], m.albedo_fuzz[1], m.albedo_fuzz[2]);
            std::memcpy(&mats[i].b.y, &inv_pr, sizeof(float));  // ref_idx: a dielectric's only
        }
        if (m.kind == RRT_MAT_DIELECTRIC && RRT_DIEL_HOST) {  // the f32 kernel's per-material constants
            float inv_eta, r0_front, r0_back;
            dielectric_consts(m.ref_idx, inv_eta, r0_front, r0_back);
            mats[i].a = make_float4(inv_eta, r0_front, r0_back, fuzz);
        }
    }
    // Spheres in BVH leaf order, each with a copy of its material record: a hit reads one
    // 32-B record at the primitive's index (no dependent material-index fetch).
    // Quads with their derived plane (quad.rs:21-37 in f64: n = cross(u, v), normal = n * (1/|n|),
    // D = dot(normal, q), w = n * (1/dot(n, n)); Vec3 / f64 is `(1/rhs) * v`, vec3.rs:142-148).
    // GQuad array: the scene's quads, media boundary quads, book-3 light quads
    std::vector<RrtQuad> light_quads;
    std::vector<rrt::GLight> glights(book3 ? ex.n_lights : 0);
    for (uint32_t l = 0; l < glights.size(); ++l) {
        const RrtLight &L = ex.lights[l];
        rrt::GLight &g = glights[l];
        g.kind = L.kind;
        g.sphere = make_float4(L.a[0], L.a[1], L.a[2], std::max(L.a[3], 0.0f));
        if (L.kind == RRT_LIGHT_QUAD) {
            RrtQuad q{};
            for (int i = 0; i < 3; ++i) q.q[i] = L.a[i], q.u[i] = L.u[i], q.v[i] = L.v[i];
            g.quad = n_quads + ex.n_bquads + (uint32_t)light_quads.size();
            const D3 n = cross(d3(L.u[0], L.u[1], L.u[2]), d3(L.v[0], L.v[1], L.v[2]));
            g.area = (float)std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);  // quad.rs:28 area = |n|
            light_quads.push_back(q);
        }
    }
    std::vector<rrt::GQuad> gquads(n_quads + (size_t)ex.n_bquads + light_quads.size());
    for (uint32_t j = 0; j < gquads.size(); ++j) {
        const RrtQuad &qd = j < n_quads ? quads[j]
                            : j < n_quads + ex.n_bquads ? ex.bquads[j - n_quads]
                                                        : light_quads[j - n_quads - ex.n_bquads];
        const D3 q = d3(qd.q[0], qd.q[1], qd.q[2]), u = d3(qd.u[0], qd.u[1], qd.u[2]), v = d3(qd.v[0], qd.v[1], qd.v[2]);
        const D3 n = cross(u, v);
        const double nn = n.x * n.x + n.y * n.y + n.z * n.z;
        const D3 normal = n * (1.0 / std::sqrt(nn));
        const double dd = normal.x * q.x + normal.y * q.y + normal.z * q.z;
        const D3 w = n * (1.0 / nn);
        rrt::GQuad &g = gquads[j];
        g.q = make_float4(qd.q[0], qd.q[1], qd.q[2], (float)dd);
        g.u = make_float4(qd.u[0], qd.u[1], qd.u[2], 0.0f);
        g.v = make_float4(qd.v[0], qd.v[1], qd.v[2], 0.0f);
        g.n = make_float4((float)normal.x, (float)normal.y, (float)normal.z, 0.0f);
        g.w = make_float4((float)w.x, (float)w.y, (float)w.z, 0.0f);
    }
    // Primitives in BVH leaf order (spheres, then quads as index n_spheres + j), each with a
    // copy of its material record: a hit reads one 32-B record at the primitive's index.
    std::vector<float4> prim_cr(n_prims);
    std::vector<rrt::GMaterial> prim_mtl(n_prims);
    std::vector<float4> prim_motion(book2 ? n_prims : 0, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (uint32_t i = 0; i < n_prims; ++i) {
        if (order[i] >= n_spheres) {  // quad j / medium j - n_quads: tagged by a negative w (spheres have r >= 0)
            const uint32_t j = order[i] - n_spheres;
            prim_cr[i] = make_float4(0.0f, 0.0f, 0.0f, -(float)(j + 1));
            prim_mtl[i] = mats[j < n_quads ? quads[j].material_index : ex.media[j - n_quads].material_index];
            if (j < n_quads) {  // the plane in the primitive and motion slots: (q, tag), (normal, D)
                const rrt::GQuad &g = gquads[j];
                prim_cr[i] = make_float4(g.q.x, g.q.y, g.q.z, -(float)(j + 1));
                prim_motion[i] = make_float4(g.n.x, g.n.y, g.n.z, g.q.w);
            }
            continue;
        }
        const RrtSphere &sp = spheres[order[i]];
        const float r = std::max(sp.center_radius[3], 0.0f);
        prim_mtl[i] = mats[sp.material_index];
        if (book2 || f64) {  // the f64 kernel forms r * r in f64 (sphere.rs:29)
            prim_cr[i] = make_float4(sp.center_radius[0], sp.center_radius[1], sp.center_radius[2], r);
        } else {  // book-1 kernel layout: r * r in the record (one multiply less per test), 1 / r in b.w
#ifndef RRT_INVR_HOST
#define RRT_INVR_HOST 1
#endif
            const volatile float r2 = r * r;  // f32, rounded once like the kernel's r * r
            const volatile float inv_r = 1.0f / r;  // the kernel's correctly rounded quotient
            const float bw = RRT_INVR_HOST ? (float)inv_r : r;
            prim_cr[i] = make_float4(sp.center_radius[0], sp.center_radius[1], sp.center_radius[2], r2);
            std::memcpy(&prim_mtl[i].b.w, &bw, sizeof(float));
        }
        if (motion) {
            const float *m = motion + 4 * (size_t)order[i];
            prim_motion[i] = make_float4(m[0], m[1], m[2], 0.0f);
        }
        if (book2 && RRT_INVR_HOST) {  // books 2 / 3: 1 / r in the motion record's w (xyz: the motion)
            const volatile float inv_r = 1.0f / r;
            prim_motion[i].w = inv_r;
        }
    }
    // Media: boundary quads follow the scene's quads in the GQuad array.
    std::vector<rrt::GMedium> gmedia(n_media);
    for (uint32_t m = 0; m < n_media; ++m) {
        const RrtMedium &md = ex.media[m];
        rrt::GMedium &g = gmedia[m];
        g.sphere = make_float4(md.sphere[0], md.sphere[1], md.sphere[2], std::max(md.sphere[3], 0.0f));
        g.kind = md.boundary_kind;
        g.first = n_quads + md.first;
        g.count = md.count;
        g.neg_inv_density = (float)(-1.0 / (double)md.density);  // constant_medium.rs:24
    }
    std::vector<rrt::GPerlin> perlin(n_perlin);
    for (uint32_t t = 0; t < n_perlin; ++t) {
        const RrtPerlin &src = ext->perlin[t];
        for (int i = 0; i < 256; ++i) {
            if (src.perm_x[i] > 255 || src.perm_y[i] > 255 || src.perm_z[i] > 255)
                return fail(RRT_E_INVALID, "Perlin permutation entry > 255");
            perlin[t].randvec[i] = make_float4(src.randvec[i][0], src.randvec[i][1], src.randvec[i][2], 0.0f);
            perlin[t].perm[i] = (uint32_t)src.perm_x[i] | ((uint32_t)src.perm_y[i] << 8) | ((uint32_t)src.perm_z[i] << 16);
        }
    }
    std::vector<rrt::GTexture> texs(n_textures);
    size_t pool = 0;
    for (uint32_t i = 0; i < n_textures; ++i) {
        const RrtTexture &t = textures[i];
        if (t.width < 0 || t.height < 0 || ((size_t)t.width * t.height > 0 && !t.rgb8))
            return fail(RRT_E_INVALID, "texture " + std::to_string(i) + " invalid");
        texs[i] = rrt::GTexture{(int32_t)pool, t.width, t.height, 0};
        pool += (size_t)t.width * t.height * 3;
    }
    if (pool > (size_t)INT32_MAX) return fail(RRT_E_INVALID, "texture pool exceeds 2 GiB");
    std::vector<uint8_t> tex_pool(pool);
    for (uint32_t i = 0; i < n_textures; ++i)
        if ((size_t)textures[i].width * textures[i].height)
            std::memcpy(tex_pool.data() + texs[i].offset, textures[i].rgb8, (size_t)textures[i].width * textures[i].height * 3);

    RrtScene *s = new RrtScene();
    s->device = device;
    s->f64 = f64;
    int rc = RRT_OK;
    do {
        if (hipSetDevice(device) != hipSuccess) { rc = fail(RRT_E_HIP, "hipSetDevice failed"); break; }
        if ((rc = upload(&s->d_nodes, fb.bytes.data(), fb.bytes.size(), "nodes"))) break;
        if ((rc = upload(&s->d_prim_cr, prim_cr.data(), prim_cr.size(), "spheres"))) break;
        if ((rc = upload(&s->d_prim_mtl, prim_mtl.data(), prim_mtl.size(), "sphere materials"))) break;
        if (book2 && (rc = upload(&s->d_prim_motion, prim_motion.data(), prim_motion.size(), "sphere motion"))) break;
        if (f64) {
            std::vector<double> inv_r(n_prims);
            for (uint32_t i = 0; i < n_prims; ++i) inv_r[i] = 1.0 / (double)prim_cr[i].w;
            if ((rc = upload(&s->d_prim_inv_r64, inv_r.data(), inv_r.size(), "sphere 1/r"))) break;
            std::vector<double4> diel(n_prims, make_double4(0.0, 0.0, 0.0, 0.0));
            for (uint32_t i = 0; i < n_prims; ++i) {
                if (prim_mtl[i].b.x != RRT_MAT_DIELECTRIC) continue;
                float eta32;
                std::memcpy(&eta32, &prim_mtl[i].b.y, sizeof(float));
                double inv_eta, r0_front, r0_back;
                dielectric_consts64((double)eta32, inv_eta, r0_front, r0_back);
                diel[i] = make_double4(inv_eta, r0_front, r0_back, 0.0);
            }
            if ((rc = upload(&s->d_prim_diel64, diel.data(), diel.size(), "dielectric constants"))) break;
        }
        if (n_perlin && (rc = upload(&s->d_perlin, perlin.data(), perlin.size(), "Perlin tables"))) break;
        if (!gquads.empty() && (rc = upload(&s->d_quads, gquads.data(), gquads.size(), "quads"))) break;
        if (n_media && (rc = upload(&s->d_media, gmedia.data(), gmedia.size(), "media"))) break;
        if (!glights.empty() && (rc = upload(&s->d_lights, glights.data(), glights.size(), "lights"))) break;
        if ((rc = upload(&s->d_tex_pool, tex_pool.data(), tex_pool.size(), "textures"))) break;
        if ((rc = upload(&s->d_texs, texs.data(), texs.size(), "texture table"))) break;
        if (hipMalloc((void **)&s->d_counters, 8 * sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc((void **)&s->d_work_counters, 8 * sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc((void **)&s->d_unit_counter, rrt::kQueues * 128u) != hipSuccess) {
            rc = fail(RRT_E_NOMEM, "hipMalloc counters failed");
            break;
        }
        if (hipMemset(s->d_counters, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
            hipMemset(s->d_work_counters, 0, 8 * sizeof(unsigned long long)) != hipSuccess) {
            rc = fail(RRT_E_HIP, "hipMemset counters failed");
            break;
        }
    } while (0);
    if (rc) {
        free_scene(s);
        return rc;
    }

    rrt::KParams &p = s->base;
    p.nodes = s->d_nodes;
    p.prim_cr = s->d_prim_cr;
    p.prim_mtl = s->d_prim_mtl;
    p.prim_inv_r64 = s->d_prim_inv_r64;
    p.prim_diel64 = s->d_prim_diel64;
    // the f64 kernel's f32 sphere pre-test (rrt_sphere32.h) holds for centers and radii within 2^20
    p.sphere32 = 0u;
    if (f64) {
        bool in = true;
        for (uint32_t i = 0; i < n_prims && in; ++i)
            for (int k = 0; k < 4; ++k) in = in && std::fabs((&prim_cr[i].x)[k]) <= 0x1.0p20f;
        p.sphere32 = in ? 1u : 0u;
        if (const char *e = std::getenv("RRT_F64_PRETEST")) p.sphere32 = p.sphere32 && std::atoi(e) != 0;
    }
    p.prim_motion = s->d_prim_motion;
    p.perlin = s->d_perlin;
    p.n_perlin = n_perlin;
    p.quads = s->d_quads;
    p.n_quads = n_quads;
    p.media = s->d_media;
    p.n_media = n_media;
    p.lights = s->d_lights;
    p.n_lights = (uint32_t)glights.size();
    p.sqrt_spp = sqrt_spp;
    p.image_tex = 0;
    for (uint32_t i = 0; i < n_materials; ++i) p.image_tex |= materials[i].kind == RRT_MAT_TEXTURED_LAMBERTIAN ? 1u : 0u;
    p.specular = 0;
    for (uint32_t i = 0; i < n_materials; ++i)
        p.specular |= materials[i].kind == RRT_MAT_METAL || materials[i].kind == RRT_MAT_DIELECTRIC ? 1u : 0u;
    p.recip_sqrt_spp = sqrt_spp ? (float)(1.0 / (double)sqrt_spp) : 0.0f;  // camera.rs:117
    p.tex_pool = s->d_tex_pool;
    p.texs = s->d_texs;
    p.counters = s->d_counters;
    const float radius = cam->params_f[0];
    for (int i = 0; i < 3; ++i) {
        p.p00[i] = cam->pixel00[i];
        p.du[i] = cam->pixel_delta_u[i];
        p.dv[i] = cam->pixel_delta_v[i];
        p.center[i] = cam->origin[i];
        p.disk_u[i] = cam->u[i] * radius;  // defocus_disk_u = u * defocus_radius (camera.rs:136-138)
        p.disk_v[i] = cam->v[i] * radius;
        p.cam_u[i] = cam->u[i];
        p.cam_v[i] = cam->v[i];
        p.background[i] = cam->background[i];
        p.cam64[0][i] = (double)cam->pixel00[i];
        p.cam64[1][i] = (double)cam->pixel_delta_u[i];
        p.cam64[2][i] = (double)cam->pixel_delta_v[i];
        p.cam64[3][i] = (double)cam->origin[i];
        p.cam64[4][i] = (double)cam->u[i] * (double)radius;  // camera.rs:136-138 in f64
        p.cam64[5][i] = (double)cam->v[i] * (double)radius;
    }
    p.defocus_radius = radius;
    p.max_depth = cam->params_u[0];
    p.seed = cam->params_u[1];
    p.bg_mode = cam->params_u[3];
    p.flags = flags;
    p.width = (uint32_t)wf;
    p.height = (uint32_t)hf;
    p.n_nodes = fb.n_nodes;
    p.n_prims = n_prims;
    p.n_unbounded = fb.n_unbounded;
    p.stack_depth = fb.stack_need;
    p.bvh_width = fb.width;
    // BVH2: the node layout already encodes the choice (80-B sign-ordered nodes are the LDS ones)
    p.scene_in_lds = fb.width == 2 ? fb.stride == (uint32_t)sizeof(rrt::GNode)
                                   : scene_lds_fit(fb.bytes.size(), n_prims, book2);
    {  // Perlin tables in LDS when the block's LDS (stack + staged scene + tables) stays within 64 KB
        // the block that launches (book-2 classes 1-3: 256 threads; book 3: 512), as launch_variant sizes it
        const bool wide = fb.n_nodes > 65535u;
        const size_t threads = (size_t)rrt::render_block_threads(book2 && !book3, wide, book3);
        const size_t stack = ((size_t)p.stack_depth * threads * (wide ? 4u : 2u) + 15u) / 16u * 16u;
        const size_t scene = p.scene_in_lds ? fb.bytes.size() + (size_t)n_prims * (rrt::kPrimBytes + (book2 ? rrt::kMotionBytes : 0)) : 0;
        p.perlin_in_lds = book2 && n_perlin > 0 &&
                          stack + scene + (size_t)n_perlin * sizeof(rrt::GPerlin) <= 64u * 1024u ? 1u : 0u;
        if (const char *e = std::getenv("RRT_PERLIN_IN_LDS")) p.perlin_in_lds = p.perlin_in_lds && std::atoi(e) != 0;
    }
    // traversal exit / leaf batch thresholds (x/256 of the live lanes), same-box sweeps against 32/32:
    // book-1 LDS scenes 56/56 (C2 +0.6 %, C4 +0.25 %); L2 scenes 64/48 (C5 +2.0 %, final_scene and
    // bouncing spheres +4 %). Book-2/3 LDS scenes by kernel class (round 6, after the class launch
    // shapes): spheres only 32/32; quads 48/48 (cornell_box +3.6 %); media 24/24 (cornell_smoke
    // +3.2 %); book 3 48/32 (+1.4 %) (profiles/r6_thresholds_sweep.log)
    {
        const int cls = book3 ? 4 : n_media ? 3 : n_quads ? 2 : 1;
        const uint32_t b2_trav = cls == 2 || cls == 4 ? 48u : cls == 3 ? 24u : 32u;
        const uint32_t b2_leaf = cls == 2 ? 48u : cls == 3 ? 24u : 32u;
        p.trav_frac = p.scene_in_lds ? (book2 ? b2_trav : 56u) : 64u;
        p.leaf_frac = p.scene_in_lds ? (book2 ? b2_leaf : 56u) : 48u;
    }
    p.min_waves = 6;
    p.chunk = accum_chunk();
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
        p.n_cus = (uint32_t)cus;
    }
    if (const char *e = std::getenv("RRT_MIN_WAVES")) p.min_waves = (uint32_t)std::atoi(e);
    p.global_waves = 7;  // L2 scenes: 256 x 7 (rrt_kernel.hip launch_width); 6 = 512 x 6, < 6 no bound
    if (const char *e = std::getenv("RRT_GLOBAL_WAVES")) p.global_waves = (uint32_t)std::atoi(e);
    if (const char *e = std::getenv("RRT_TRAV_FRAC")) p.trav_frac = (uint32_t)std::min(256, std::max(0, std::atoi(e)));
    if (const char *e = std::getenv("RRT_LEAF_FRAC")) p.leaf_frac = (uint32_t)std::min(256, std::max(0, std::atoi(e)));

    RrtBvhInfo &bi = s->info;
    bi.n_nodes = fb.n_nodes;
    bi.n_leaves = fb.n_leaves;
    bi.max_depth = fb.max_depth;
    bi.max_leaf_size = fb.max_leaf;
    bi.node_bytes = fb.bytes.size();
    bi.node_stride = fb.stride;
    bi.width = fb.width;
    bi.max_leaf_param = max_leaf;
    bi.n_unbounded = fb.n_unbounded;
    bi.prim_bytes = (uint64_t)n_prims * (rrt::kPrimBytes + (book2 ? rrt::kMotionBytes : 0)) +
                    (uint64_t)gquads.size() * sizeof(rrt::GQuad) + (uint64_t)n_media * sizeof(rrt::GMedium);
    *out = s;
    return RRT_OK;
}

extern "C" {

int32_t rrt_scene_create(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                         const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                         uint32_t n_textures, uint32_t flags, int32_t device, RrtScene **out) {
    return scene_create(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, nullptr, flags, device,
                        out);
}

int32_t rrt_scene_create_ex(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                            uint32_t n_textures, const RrtSceneExt *ext, uint32_t flags, int32_t device,
                            RrtScene **out) {
    return scene_create(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, ext, flags, device,
                        out);
}

int32_t rrt_build_bvh(const RrtSphere *spheres, uint32_t n_spheres, uint32_t width, uint32_t max_leaf,
                      void *nodes_out, size_t nodes_cap, uint32_t *prim_order_out, RrtBvhInfo *info) {
    return rrt_build_bvh_ex(spheres, n_spheres, nullptr, width, max_leaf, nodes_out, nodes_cap, prim_order_out, info);
}

int32_t rrt_build_bvh_ex(const RrtSphere *spheres, uint32_t n_spheres, const RrtSceneExt *ext, uint32_t width,
                         uint32_t max_leaf, void *nodes_out, size_t nodes_cap, uint32_t *prim_order_out,
                         RrtBvhInfo *info) {
    if (n_spheres && !spheres) return fail(RRT_E_INVALID, "null spheres");
    const ExtView ex(ext);
    for (uint32_t m = 0; m < ex.n_media; ++m)
        if (ex.media[m].boundary_kind == RRT_BOUNDARY_QUADS &&
            (ex.media[m].count == 0 || (uint64_t)ex.media[m].first + ex.media[m].count > ex.n_bquads))
            return fail(RRT_E_INVALID, "medium " + std::to_string(m) + ": boundary quad range out of bounds");
    uint32_t dw, dl;
    bvh_defaults(dw, dl);
    if (width == 0) width = dw;
    if (max_leaf == 0) max_leaf = dl;
    if ((width != 2 && width != 4) || max_leaf > (width == 2 ? rrt::kMaxLeafPrims : 15u))
        return fail(RRT_E_INVALID, "width must be 2 or 4, max_leaf <= 7 (width 2) or 15 (width 4)");
    std::vector<uint32_t> order;
    // the tree and layout scene creation would pick (scene_bvh), except that scene creation's
    // book-2 test also counts book-2 materials, whose motion bytes can tip the LDS fit of a scene
    // with such materials and no book-2 geometry (then the node price and the tree differ too)
    const bool book2 = ex.motion || ex.n_quads || ex.n_media;
    const FlatBvh fb = scene_bvh(spheres, n_spheres, ex, width, max_leaf, book2, false, order);
    if (info) {
        *info = RrtBvhInfo{};
        info->n_nodes = fb.n_nodes;
        info->n_leaves = fb.n_leaves;
        info->max_depth = fb.max_depth;
        info->max_leaf_size = fb.max_leaf;
        info->node_bytes = fb.bytes.size();
        info->node_stride = fb.stride;
        info->prim_bytes = (uint64_t)order.size() * (rrt::kPrimBytes + (book2 ? rrt::kMotionBytes : 0)) +
                           ((uint64_t)ex.n_quads + ex.n_bquads) * sizeof(rrt::GQuad) +
                           (uint64_t)ex.n_media * sizeof(rrt::GMedium);
        info->width = fb.width;
        info->max_leaf_param = max_leaf;
        info->n_unbounded = fb.n_unbounded;
    }
    if (nodes_cap == 0) return RRT_OK;
    if (!nodes_out || nodes_cap < fb.bytes.size() || (order.size() && !prim_order_out))
        return fail(RRT_E_INVALID, "nodes buffer too small (need " + std::to_string(fb.bytes.size()) + " bytes)");
    std::memcpy(nodes_out, fb.bytes.data(), fb.bytes.size());
    if (order.size()) std::memcpy(prim_order_out, order.data(), order.size() * sizeof(uint32_t));
    return RRT_OK;
}

int32_t rrt_scene_destroy(RrtScene *scene) {
    free_scene(scene);
    return RRT_OK;
}

int32_t rrt_scene_bvh_info(const RrtScene *scene, RrtBvhInfo *out) {
    if (!scene || !out) return fail(RRT_E_INVALID, "null scene or out");
    *out = scene->info;
    return RRT_OK;
}

int32_t rrt_tile_rows(uint32_t height, const RrtTile *tile, uint32_t *rows_out) {
    if (int rc = check_tile_shape(tile)) return rc;
    if (!rows_out) return fail(RRT_E_INVALID, "null rows_out");
    *rows_out = tile_rows_of(height, *tile);
    return RRT_OK;
}

int32_t rrt_tile_row_index(uint32_t height, const RrtTile *tile, uint32_t local_row, uint32_t *row_out) {
    if (int rc = check_tile_shape(tile)) return rc;
    if (!row_out) return fail(RRT_E_INVALID, "null row_out");
    if (local_row >= tile_rows_of(height, *tile)) return fail(RRT_E_INVALID, "local_row out of range");
    const uint32_t band = local_row / tile->band_rows;
    *row_out = (band * tile->n_ranks + band_slot(*tile, band)) * tile->band_rows + local_row % tile->band_rows;
    return RRT_OK;
}

// The tile's render into d_accum (float4 rows) or, for an f64 scene, d_accum64 (D4 rows; a float
// d_accum then receives the f64 sums rounded to f32 from the scene's own f64 buffer).
static int32_t render_tile(RrtScene *scene, const RrtTile *tile, float *d_accum, rrt::D4 *d_accum64, void *stream) {
    if (int rc = check_tile(scene, tile)) return rc;
    rrt::KParams p;
    if (int rc = fill_params(scene, tile, d_accum, p)) return rc;
    if (p.tile_rows && !d_accum && !d_accum64) return fail(RRT_E_INVALID, "null d_accum");
    HIP_TRY(hipSetDevice(scene->device), "hipSetDevice");
    const size_t n_px = (size_t)p.tile_rows * p.width;
    if (scene->f64) {
        p.accum64 = d_accum64;
        if (!d_accum64 && n_px > scene->accum64_cap) {  // float output: the f64 sums go to the scene's buffer first
            (void)hipFree(scene->d_accum64);
            scene->d_accum64 = nullptr;
            scene->accum64_cap = 0;
            HIP_TRY(hipMalloc((void **)&scene->d_accum64, n_px * sizeof(rrt::D4)), "hipMalloc f64 accum");
            scene->accum64_cap = n_px;
        }
        if (!d_accum64) p.accum64 = scene->d_accum64;
    }
    if (p.n_chunks == 0) {  // no samples: accum = 0 (sums and count)
        if (d_accum)
            HIP_TRY(hipMemsetAsync(d_accum, 0, n_px * sizeof(float4), (hipStream_t)stream), "hipMemsetAsync accum");
        if (d_accum64)
            HIP_TRY(hipMemsetAsync(d_accum64, 0, n_px * sizeof(rrt::D4), (hipStream_t)stream), "hipMemsetAsync accum");
        return RRT_OK;
    }
    HIP_TRY(rrt::launch_render(p, (hipStream_t)stream), "render kernel launch");
    if (scene->f64 && d_accum)
        HIP_TRY(rrt::launch_accum64_to_f32(p.accum64, reinterpret_cast<float4 *>(d_accum), (uint32_t)n_px,
                                           (hipStream_t)stream),
                "f64 accum conversion launch");
    const uint32_t per_pass = (p.pass_chunks == 0 || p.pass_chunks >= p.n_chunks) ? p.n_chunks : p.pass_chunks;
    scene->last_passes = (p.n_chunks + per_pass - 1) / per_pass;
    scene->last_groups = p.n_work_tiles * per_pass;
    return RRT_OK;
}

int32_t rrt_render_tile_async(RrtScene *scene, const RrtTile *tile, float *d_accum, void *stream) {
    return render_tile(scene, tile, d_accum, nullptr, stream);
}

int32_t rrt_render_tile_f64_async(RrtScene *scene, const RrtTile *tile, double *d_accum, void *stream) {
    if (scene && !scene->f64) return fail(RRT_E_INVALID, "rrt_render_tile_f64_async: scene not created with RRT_FLAG_F64");
    return render_tile(scene, tile, nullptr, reinterpret_cast<rrt::D4 *>(d_accum), stream);
}

namespace {
// Progress of a render in flight on `scene`'s device (the one-shot call): the work queues' heads
// read on a side stream while the kernel runs. Head q counts the claims of queue q (group g =
// claim * kQueues + q), capped at the queue's groups; a pass boundary resets the heads. Returns
// the fraction in [0, 1), or -1 when the heads cannot be read.
double render_progress(RrtScene *scene, hipStream_t side, uint32_t *host_heads, uint32_t &pass, uint32_t &last_sum) {
    if (hipMemcpyAsync(host_heads, scene->d_unit_counter, rrt::kQueues * 128u, hipMemcpyDeviceToHost, side) != hipSuccess ||
        hipStreamSynchronize(side) != hipSuccess)
        return -1.0;
    const uint32_t groups = scene->last_groups, passes = std::max(1u, scene->last_passes);
    uint32_t sum = 0;
    for (uint32_t q = 0; q < rrt::kQueues; ++q) {
        const uint32_t mine = groups > q ? (groups - q + rrt::kQueues - 1) / rrt::kQueues : 0u;
        sum += std::min(host_heads[32u * q], mine);
    }
    if (sum + groups / 4 < last_sum && pass + 1 < passes) ++pass;  // the heads were reset: next pass
    last_sum = sum;
    const double in_pass = groups ? (double)sum / groups : 0.0;
    return std::min(0.999, (pass + in_pass) / passes);
}
}  // namespace

int32_t rrt_scene_read_counters(RrtScene *scene, RrtCounters *out) {
    if (!scene || !out) return fail(RRT_E_INVALID, "null scene or out");
    unsigned long long c[8];
    HIP_TRY(hipSetDevice(scene->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(hipMemcpy(c, scene->d_counters, sizeof(c), hipMemcpyDeviceToHost), "copy counters");
    *out = RrtCounters{c[0], c[1], c[2], c[3], c[4]};
    return RRT_OK;
}

int32_t rrt_scene_reset_counters(RrtScene *scene) {
    if (!scene) return fail(RRT_E_INVALID, "null scene");
    HIP_TRY(hipSetDevice(scene->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(hipMemset(scene->d_counters, 0, 8 * sizeof(unsigned long long)), "reset counters");
    return RRT_OK;
}

int32_t rrt_scene_count_work(RrtScene *scene, const RrtTile *tile, RrtCounters *out) {
    if (int rc = check_tile(scene, tile)) return rc;
    if (!out) return fail(RRT_E_INVALID, "null out");
    rrt::KParams p;
    if (int rc = fill_params(scene, tile, nullptr, p)) return rc;
    HIP_TRY(hipSetDevice(scene->device), "hipSetDevice");
    float4 *scratch = nullptr;
    const size_t elem = scene->f64 ? sizeof(rrt::D4) : sizeof(float4);
    HIP_TRY(hipMalloc((void **)&scratch, std::max<size_t>((size_t)p.tile_rows * p.width, 1) * elem),
            "hipMalloc scratch accum");
    p.accum = scratch;
    p.accum64 = reinterpret_cast<rrt::D4 *>(scratch);
    p.counters = scene->d_work_counters;
    hipError_t e = hipMemset(scene->d_work_counters, 0, 8 * sizeof(unsigned long long));
    if (e == hipSuccess) e = rrt::launch_render_counting(p, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long c[8] = {0};
    if (e == hipSuccess) e = hipMemcpy(c, scene->d_work_counters, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipFree(scratch);
    if (e != hipSuccess) return fail(RRT_E_HIP, std::string("counting render failed: ") + hipGetErrorString(e));
    *out = RrtCounters{c[0], c[1], c[2], c[3], c[4]};
    return RRT_OK;
}

// ---- one-shot drop-in (cuda/mod.rs:342-439) ---------------------------------------------
}  // extern "C"

// Test mode (rrt_testing_device_wrap(1), a test-only entry point; no environment variable reaches
// it): worker g of a one-shot render runs on device g % device_count, so the multi-device path
// (threads, row bands, the strided copies into the caller's image) runs with n_gpus > 1 on a
// one-GPU box (tests/test_gpu_multidevice.py). Off by default: n_gpus must not exceed the visible
// devices.
static std::atomic<bool> g_device_wrap{false};
extern "C" void rrt_testing_device_wrap(int32_t on) { g_device_wrap.store(on != 0); }

// Test mode (rrt_testing_f64_layout, a test-only entry point): the f64 kernel stages a scene that fits
// the block's LDS in the given layout instead of its automatic choice (every layout renders the same
// bits; tests/test_gpu_books64.py reaches each fallback with it). -1 restores the automatic choice.
extern "C" void rrt_testing_f64_layout(int32_t layout) { rrt::set_f64_layout(layout); }

extern "C" int32_t rrt_testing_recip_check(uint64_t *mismatches) {
    if (!mismatches) return fail(RRT_E_INVALID, "null mismatches");
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, 3 * sizeof(unsigned long long)), "hipMalloc");
    hipError_t e = hipMemset(d, 0, 3 * sizeof(unsigned long long));
    if (e == hipSuccess) e = rrt::launch_recip_check(d, nullptr);
    unsigned long long h[3] = {0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RRT_E_HIP, std::string("rrt_testing_recip_check: ") + hipGetErrorString(e));
    for (int i = 0; i < 3; ++i) mismatches[i] = h[i];
    return RRT_OK;
}
extern "C" int32_t rrt_testing_sqrt64_check(uint64_t *out) {
    if (!out) return fail(RRT_E_INVALID, "null out");
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, 2 * sizeof(unsigned long long)), "hipMalloc");
    hipError_t e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = rrt::launch_sqrt64_check(d, nullptr);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RRT_E_HIP, std::string("rrt_testing_sqrt64_check: ") + hipGetErrorString(e));
    out[0] = h[0];
    out[1] = h[1];
    return RRT_OK;
}
extern "C" int32_t rrt_testing_trig32_check(double *out) {
    if (!out) return fail(RRT_E_INVALID, "null out");
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, 2 * sizeof(unsigned long long)), "hipMalloc");
    hipError_t e = hipMemset(d, 0, 2 * sizeof(unsigned long long));
    double bounds[2] = {0.0, 0.0};
    if (e == hipSuccess) e = rrt::launch_trig32_check(d, bounds, nullptr);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RRT_E_HIP, std::string("rrt_testing_trig32_check: ") + hipGetErrorString(e));
    std::memcpy(&out[0], &h[0], sizeof(double));
    std::memcpy(&out[1], &h[1], sizeof(double));
    out[2] = bounds[0];
    out[3] = bounds[1];
    return RRT_OK;
}
static bool device_wrap() { return g_device_wrap.load(); }

// One-shot frame on n_gpus devices: float accum rows (accum_out), f64 accum rows (accum64_out, the
// RRT_FLAG_F64 kernel) or render_io-quantised rows (rgb8_out, quantised on the device) assembled
// into the caller's image.
static int32_t render_frame(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                            uint32_t n_textures, const RrtSceneExt *ext, uint32_t total_spp, uint32_t n_gpus,
                            uint32_t flags, float *accum_out, uint8_t *rgb8_out, double *accum64_out = nullptr) {
    if (!cam || (!accum_out && !rgb8_out && !accum64_out)) return fail(RRT_E_INVALID, "null camera or output buffer");
    if (accum64_out) flags |= RRT_FLAG_F64;
    if (total_spp == 0) total_spp = (uint32_t)std::max(cam->params_f[3], 1.0f);  // cuda/mod.rs:384
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RRT_E_NODEV, "no HIP device available");
    if (n_gpus == 0) n_gpus = 1;
    const bool wrap = device_wrap();
    if ((int)n_gpus > ndev && !wrap)
        return fail(RRT_E_INVALID, "n_gpus=" + std::to_string(n_gpus) + " > visible devices " + std::to_string(ndev));
    if (n_gpus > 64) return fail(RRT_E_INVALID, "n_gpus > 64");
    const uint32_t width = (uint32_t)cam->params_f[1];
    const uint32_t height = (uint32_t)cam->params_f[2];

    std::mutex mu;
    std::string first_err;
    int first_rc = RRT_OK;
    std::atomic<uint32_t> done{0};
    std::vector<double> frac(n_gpus, 0.0);  // per-GPU progress (guarded by mu)
    auto worker = [&](uint32_t g) {
        auto set_err = [&](int rc) {
            std::lock_guard<std::mutex> lk(mu);
            if (first_rc == RRT_OK) {
                first_rc = rc;
                first_err = g_err;
            }
        };
        RrtScene *scene = nullptr;
        int rc = scene_create(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, ext, flags,
                              (int32_t)(g % (uint32_t)ndev), &scene);
        if (rc) return set_err(rc);
        const RrtTile tile{16u, g, n_gpus, 0u, total_spp};
        const uint32_t rows = tile_rows_of(height, tile);
        const size_t n_px = (size_t)rows * width;
        const size_t px_bytes = accum64_out ? sizeof(rrt::D4) : sizeof(float4);
        const size_t row_bytes = rgb8_out ? (size_t)width * 3 : (size_t)width * px_bytes;
        float *d_accum = nullptr;
        uint8_t *d_rgb8 = nullptr;
        hipError_t e = hipMalloc((void **)&d_accum, std::max<size_t>(n_px, 1) * px_bytes);
        if (e == hipSuccess && rgb8_out) e = hipMalloc((void **)&d_rgb8, std::max<size_t>(n_px, 1) * 3);
        if (e != hipSuccess) {
            (void)hipFree(d_accum);
            rrt_scene_destroy(scene);
            g_err = std::string("hipMalloc output failed: ") + hipGetErrorString(e);
            return set_err(RRT_E_NOMEM);
        }
        rc = accum64_out ? rrt_render_tile_f64_async(scene, &tile, reinterpret_cast<double *>(d_accum), nullptr)
                         : rrt_render_tile_async(scene, &tile, d_accum, nullptr);
        if (!rc && !(flags & RRT_FLAG_QUIET)) {
            // within-GPU progress (the reference prints one line per sample pass, cuda/mod.rs:426-431):
            // poll the work-queue heads every 100 ms while the kernel runs
            hipEvent_t ev = nullptr;
            hipStream_t side = nullptr;
            uint32_t *heads = nullptr;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(ev, nullptr) == hipSuccess &&
                hipStreamCreateWithFlags(&side, hipStreamNonBlocking) == hipSuccess &&
                hipHostMalloc((void **)&heads, rrt::kQueues * 128u, 0) == hipSuccess) {
                uint32_t pass = 0, last_sum = 0;
                int shown = -1;
                // the end of the render is noticed within ~1 ms (a 100-ms sleep rounded a one-shot
                // call up to the next tick: an 89-ms C2 frame took >= 100 ms); the heads are read
                // every 100 ms
                auto next_read = std::chrono::steady_clock::now() + std::chrono::milliseconds(100);
                while (hipEventQuery(ev) == hipErrorNotReady) {
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                    if (std::chrono::steady_clock::now() < next_read) continue;
                    next_read += std::chrono::milliseconds(100);
                    const double f = render_progress(scene, side, heads, pass, last_sum);
                    if (f < 0.0) break;
                    std::lock_guard<std::mutex> lk(mu);
                    frac[g] = f;
                    double all = 0.0;
                    for (double x : frac) all += x;
                    const int pct = (int)(100.0 * all / n_gpus);
                    if (pct != shown) {
                        shown = pct;
                        std::fprintf(stderr, "\rHIP progress: %d%% (%u/%u GPUs done)", pct, done.load(), n_gpus);
                    }
                }
            }
            if (heads) (void)hipHostFree(heads);
            if (side) (void)hipStreamDestroy(side);
            if (ev) (void)hipEventDestroy(ev);
        }
        if (!rc && rgb8_out) {
            const float scale = 1.0f / (float)total_spp;  // render_io.rs:10
            e = rrt::launch_quantize(d_accum, d_rgb8, (uint32_t)n_px, scale, nullptr);
            if (e != hipSuccess) {
                g_err = std::string("quantise launch failed: ") + hipGetErrorString(e);
                rc = RRT_E_HIP;
            }
        }
        if (!rc && rows) {
            // straight into the caller's image: the tile's local bands (band_rows rows each) are
            // contiguous on both sides, so two strided 2-D copies place every whole band — the
            // even local bands j (image band j * n_ranks + rank) and the odd ones (image band
            // j * n_ranks + n_ranks - 1 - rank), each at a stride of two periods — and one plain
            // copy the partial last band
            const uint8_t *src = rgb8_out ? (const uint8_t *)d_rgb8 : (const uint8_t *)d_accum;
            uint8_t *dst = rgb8_out ? rgb8_out
                                    : accum64_out ? reinterpret_cast<uint8_t *>(accum64_out) : reinterpret_cast<uint8_t *>(accum_out);
            const size_t band_bytes = (size_t)tile.band_rows * row_bytes;
            const uint32_t whole = rows / tile.band_rows, rest = rows % tile.band_rows;
            e = hipDeviceSynchronize();
            for (uint32_t par = 0; par < 2 && e == hipSuccess; ++par) {
                const uint32_t count = (whole + 1u - par) / 2u;  // local bands j = par, par + 2, ...
                if (count)
                    e = hipMemcpy2D(dst + ((size_t)par * tile.n_ranks + band_slot(tile, par)) * band_bytes,
                                    band_bytes * 2u * tile.n_ranks, src + (size_t)par * band_bytes, 2u * band_bytes,
                                    band_bytes, count, hipMemcpyDeviceToHost);
            }
            if (e == hipSuccess && rest)
                e = hipMemcpy(dst + ((size_t)whole * tile.n_ranks + band_slot(tile, whole)) * band_bytes,
                              src + (size_t)whole * band_bytes, (size_t)rest * row_bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                g_err = std::string("render failed: ") + hipGetErrorString(e);
                rc = RRT_E_HIP;
            }
        }
        (void)hipFree(d_accum);
        (void)hipFree(d_rgb8);
        rrt_scene_destroy(scene);
        if (rc) return set_err(rc);
        const uint32_t d = ++done;
        if (!(flags & RRT_FLAG_QUIET)) {
            std::lock_guard<std::mutex> lk(mu);
            frac[g] = 1.0;
            double all = 0.0;
            for (double x : frac) all += x;
            std::fprintf(stderr, "\rHIP progress: %d%% (%u/%u GPUs done)", (int)(100.0 * all / n_gpus), d, n_gpus);
            if (d == n_gpus) std::fprintf(stderr, "\n");
        }
    };
    if (n_gpus == 1) {
        worker(0);
    } else {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < n_gpus; ++g) th.emplace_back(worker, g);
        for (auto &t : th) t.join();
    }
    if (first_rc) return fail(first_rc, first_err);
    return RRT_OK;
}

extern "C" {

int32_t rrt_hip_render(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                       const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                       uint32_t n_textures, uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                       float *accum_out) {
    if (!accum_out) return fail(RRT_E_INVALID, "null camera or accum_out");
    return render_frame(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, nullptr, total_spp,
                        n_gpus, flags, accum_out, nullptr);
}

int32_t rrt_hip_render_ex(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                          const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                          uint32_t n_textures, const RrtSceneExt *ext, uint32_t total_spp, uint32_t n_gpus,
                          uint32_t flags, float *accum_out) {
    if (!accum_out) return fail(RRT_E_INVALID, "null camera or accum_out");
    return render_frame(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, ext, total_spp,
                        n_gpus, flags, accum_out, nullptr);
}

int32_t rrt_hip_render_f64(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                           const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                           uint32_t n_textures, uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                           double *accum_out) {
    if (!accum_out) return fail(RRT_E_INVALID, "null camera or accum_out");
    return render_frame(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, nullptr, total_spp,
                        n_gpus, flags | RRT_FLAG_F64, nullptr, nullptr, accum_out);
}

int32_t rrt_hip_render_rgb8(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                            const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                            uint32_t n_textures, uint32_t total_spp, uint32_t n_gpus, uint32_t flags,
                            uint8_t *rgb8_out) {
    if (!rgb8_out) return fail(RRT_E_INVALID, "null camera or rgb8_out");
    return render_frame(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, nullptr, total_spp,
                        n_gpus, flags, nullptr, rgb8_out);
}

int32_t rrt_hip_render_rgb8_ex(const RrtCamera *cam, const RrtSphere *spheres, uint32_t n_spheres,
                               const RrtMaterial *materials, uint32_t n_materials, const RrtTexture *textures,
                               uint32_t n_textures, const RrtSceneExt *ext, uint32_t total_spp, uint32_t n_gpus,
                               uint32_t flags, uint8_t *rgb8_out) {
    if (!rgb8_out) return fail(RRT_E_INVALID, "null camera or rgb8_out");
    return render_frame(cam, spheres, n_spheres, materials, n_materials, textures, n_textures, ext, total_spp,
                        n_gpus, flags, nullptr, rgb8_out);
}

int32_t rrt_quantize_accum_async(uint32_t n_pixels, const float *d_accum, uint32_t samples_per_pixel, uint8_t *d_rgb8,
                                 void *stream) {
    if (n_pixels && (!d_accum || !d_rgb8)) return fail(RRT_E_INVALID, "null d_accum or d_rgb8");
    const float scale = samples_per_pixel > 0 ? 1.0f / (float)samples_per_pixel : 0.0f;
    const hipError_t e = rrt::launch_quantize(d_accum, d_rgb8, n_pixels, scale, (hipStream_t)stream);
    if (e != hipSuccess) return fail(RRT_E_HIP, std::string("quantise launch failed: ") + hipGetErrorString(e));
    return RRT_OK;
}

// ---- scene builder (gpu/mod.rs:124-301) ------------------------------------------------
int32_t rrt_apply_overrides(const RrtOverrides *o, int32_t book, double *aspect_ratio, int32_t *image_width,
                            int32_t *samples_per_pixel, int32_t *max_depth, double *vfov, double *lookfrom,
                            double *lookat, double *vup, double *defocus_angle, double *focus_dist,
                            double *background, int32_t *has_background) {
    if (!o) return RRT_OK;
    if (o->has_aspect_ratio && aspect_ratio) *aspect_ratio = o->aspect_ratio;
    if (o->has_image_width && image_width) *image_width = o->image_width;
    if (o->has_samples_per_pixel && samples_per_pixel) *samples_per_pixel = o->samples_per_pixel;
    if (o->has_max_depth && max_depth) *max_depth = o->max_depth;
    if (o->has_vfov && vfov) *vfov = o->vfov;
    if (o->has_lookfrom && lookfrom) std::memcpy(lookfrom, o->lookfrom, 24);
    if (o->has_lookat && lookat) std::memcpy(lookat, o->lookat, 24);
    if (o->has_vup && vup) std::memcpy(vup, o->vup, 24);
    if (o->has_defocus_angle && defocus_angle) *defocus_angle = o->defocus_angle;
    if (o->has_focus_dist && focus_dist) *focus_dist = o->focus_dist;
    // book 1 ignores `background` (in_one_weekend/mod.rs:23-55); book 2 and the GPU
    // scene builder apply it (the_next_week/mod.rs:62-64, gpu/mod.rs:169-172).
    if (book != 1 && o->has_background && background) {
        std::memcpy(background, o->background, 24);
        if (has_background) *has_background = 1;
    }
    return RRT_OK;
}

int32_t rrt_make_camera(double aspect_ratio, int32_t image_width, int32_t samples_per_pixel, int32_t max_depth,
                        double vfov, const double *lookfrom_, const double *lookat_, const double *vup_,
                        double defocus_angle, double focus_dist, const double *background, uint32_t sample_seed,
                        uint32_t n_spheres, RrtCamera *cam) {
    if (!lookfrom_ || !lookat_ || !vup_ || !cam) return fail(RRT_E_INVALID, "null camera argument");
    if (image_width < 1) return fail(RRT_E_INVALID, "image_width must be >= 1");
    int32_t image_height = (int32_t)((double)image_width / aspect_ratio);  // gpu/mod.rs:174-177
    if (image_height < 1) image_height = 1;
    const D3 lookfrom = d3(lookfrom_[0], lookfrom_[1], lookfrom_[2]);
    const D3 lookat = d3(lookat_[0], lookat_[1], lookat_[2]);
    const D3 vup = d3(vup_[0], vup_[1], vup_[2]);
    const double theta = degrees_to_radians(vfov);
    const double h = std::tan(theta / 2.0);
    const double viewport_height = 2.0 * h * focus_dist;
    const double viewport_width = viewport_height * ((double)image_width / (double)image_height);
    const D3 w = unit_vector(lookfrom - lookat);
    const D3 u = unit_vector(cross(vup, w));
    const D3 v = cross(w, u);
    const D3 viewport_u = u * viewport_width;
    const D3 viewport_v = v * -viewport_height;
    const D3 pixel_delta_u = viewport_u / (double)image_width;
    const D3 pixel_delta_v = viewport_v / (double)image_height;
    const D3 upper_left = lookfrom - (w * focus_dist) - viewport_u / 2.0 - viewport_v / 2.0;
    const D3 pixel00 = upper_left + (pixel_delta_u + pixel_delta_v) * 0.5;
    const double defocus_radius = focus_dist * std::tan(degrees_to_radians(defocus_angle / 2.0));

    std::memset(cam, 0, sizeof(*cam));
    put4(cam->origin, (float)lookfrom.x, (float)lookfrom.y, (float)lookfrom.z, 0.0f);
    put4(cam->pixel00, (float)pixel00.x, (float)pixel00.y, (float)pixel00.z, 0.0f);
    put4(cam->pixel_delta_u, (float)pixel_delta_u.x, (float)pixel_delta_u.y, (float)pixel_delta_u.z, 0.0f);
    put4(cam->pixel_delta_v, (float)pixel_delta_v.x, (float)pixel_delta_v.y, (float)pixel_delta_v.z, 0.0f);
    put4(cam->u, (float)u.x, (float)u.y, (float)u.z, 0.0f);
    put4(cam->v, (float)v.x, (float)v.y, (float)v.z, 0.0f);
    if (background) put4(cam->background, (float)background[0], (float)background[1], (float)background[2], 0.0f);
    put4(cam->params_f, (float)defocus_radius, (float)image_width, (float)image_height, (float)samples_per_pixel);
    cam->params_u[0] = (uint32_t)max_depth;
    cam->params_u[1] = sample_seed;
    cam->params_u[2] = n_spheres;
    cam->params_u[3] = background ? 1u : 0u;
    return RRT_OK;
}

int32_t rrt_build_in_one_weekend_scene(const RrtOverrides *ov, uint64_t seed, int32_t grid_half, RrtCamera *cam,
                                       RrtSphere *spheres, RrtMaterial *materials, uint32_t sphere_cap,
                                       uint32_t *n_spheres) {
    if (!n_spheres) return fail(RRT_E_INVALID, "null n_spheres");
    if (grid_half < 0 || grid_half > 1000) return fail(RRT_E_INVALID, "grid_half out of range");
    double aspect_ratio = 16.0 / 9.0;
    int32_t image_width = 1200, samples_per_pixel = 10, max_depth = 20;
    double vfov = 20.0;
    double lookfrom[3] = {13.0, 2.0, 3.0}, lookat[3] = {0.0, 0.0, 0.0}, vup[3] = {0.0, 1.0, 0.0};
    double defocus_angle = 0.6, focus_dist = 10.0;
    double background[3] = {0.0, 0.0, 0.0};
    int32_t has_bg = 0;
    rrt_apply_overrides(ov, 0, &aspect_ratio, &image_width, &samples_per_pixel, &max_depth, &vfov, lookfrom, lookat,
                        vup, &defocus_angle, &focus_dist, background, &has_bg);

    std::vector<RrtSphere> sph;
    std::vector<RrtMaterial> mat;
    auto add_material = [&](uint32_t kind, float r, float g, float b, float fuzz, float ref_idx) {
        RrtMaterial m{};
        put4(m.albedo_fuzz, r, g, b, fuzz);
        m.kind = kind;
        m.ref_idx = ref_idx;
        mat.push_back(m);
        return (uint32_t)(mat.size() - 1);
    };
    auto add_sphere = [&](float x, float y, float z, float r, uint32_t m) {
        RrtSphere s{};
        put4(s.center_radius, x, y, z, r);
        s.material_index = m;
        sph.push_back(s);
    };
    SmallRng rng(seed);
    add_sphere(0.0f, -1000.0f, 0.0f, 1000.0f, add_material(0, 0.5f, 0.5f, 0.5f, 0.0f, 1.0f));
    for (int a = -grid_half; a < grid_half; ++a) {
        for (int b = -grid_half; b < grid_half; ++b) {
            const float choose_mat = rng.gen_f32();
            const double cx = (double)a + 0.9 * rng.gen_f64();
            const double cz = (double)b + 0.9 * rng.gen_f64();
            const D3 center = d3(cx, 0.2, cz);
            if (length(center - d3(4.0, 0.2, 0.0)) > 0.9) {
                uint32_t m;
                if (choose_mat < 0.8f) {
                    float alb[3];
                    for (int c = 0; c < 3; ++c) {
                        const float p = rng.gen_f32();
                        const float q = rng.gen_f32();
                        alb[c] = p * q;
                    }
                    m = add_material(0, alb[0], alb[1], alb[2], 0.0f, 1.0f);
                } else if (choose_mat < 0.95f) {
                    float alb[3];
                    for (int c = 0; c < 3; ++c) alb[c] = rng.gen_range_f32(0.5f, 1.0f);
                    const float fuzz = rng.gen_f32() * 0.5f;
                    m = add_material(1, alb[0], alb[1], alb[2], fuzz, 1.0f);
                } else {
                    m = add_material(2, 1.0f, 1.0f, 1.0f, 0.0f, 1.5f);
                }
                add_sphere((float)center.x, (float)center.y, (float)center.z, 0.2f, m);
            }
        }
    }
    add_sphere(0.0f, 1.0f, 0.0f, 1.0f, add_material(2, 1.0f, 1.0f, 1.0f, 0.0f, 1.5f));
    add_sphere(-4.0f, 1.0f, 0.0f, 1.0f, add_material(0, 0.4f, 0.2f, 0.1f, 0.0f, 1.0f));
    add_sphere(4.0f, 1.0f, 0.0f, 1.0f, add_material(1, 0.7f, 0.6f, 0.5f, 0.0f, 1.0f));
    const uint32_t sample_seed = rng.next_u32();

    *n_spheres = (uint32_t)sph.size();
    if (cam) {
        int rc = rrt_make_camera(aspect_ratio, image_width, samples_per_pixel, max_depth, vfov, lookfrom, lookat, vup,
                                 defocus_angle, focus_dist, has_bg ? background : nullptr, sample_seed,
                                 (uint32_t)sph.size(), cam);
        if (rc) return rc;
    }
    if (sphere_cap == 0) return RRT_OK;
    if (sphere_cap < sph.size() || !spheres || !materials)
        return fail(RRT_E_INVALID, "sphere_cap too small (need " + std::to_string(sph.size()) + ")");
    std::memcpy(spheres, sph.data(), sph.size() * sizeof(RrtSphere));
    std::memcpy(materials, mat.data(), mat.size() * sizeof(RrtMaterial));
    return RRT_OK;
}

// ---- book-2 scenes (the_next_week/mod.rs:83-255) -----------------------------------------
// The reference draws from the thread-local entropy RNG (rtweekend.rs:9-30); here the same
// draws, in the same order, come from SmallRng(seed): random_double() = gen_range(0.0..1.0),
// random_double_range = gen_range(min..max), random_int(min,max) = random_double_range(min,
// max+1) as i32 (rtweekend.rs:17-30). Parity unpinned (entropy RNG).
// Book-2 scenes 1..10 and the book-3 scene (kBook3Scene), flattened into RrtBookScene.
static const int32_t kBook3Scene = 100;
static int32_t build_book_scene(int32_t scene, const RrtOverrides *ov, uint64_t seed, RrtBookScene *out) {
    if (!out) return fail(RRT_E_INVALID, "null output");
    // Camera (the_next_week/mod.rs:137-150, 177-190, 203-216, 237-250)
    double aspect_ratio = 16.0 / 9.0;
    int32_t image_width = 400, samples_per_pixel = 100, max_depth = 50;
    double vfov = 20.0;
    double lookfrom[3] = {13.0, 2.0, 3.0}, lookat[3] = {0.0, 0.0, 0.0}, vup[3] = {0.0, 1.0, 0.0};
    double defocus_angle = 0.0, focus_dist = 10.0;
    double background[3] = {0.70, 0.80, 1.00};
    int32_t has_bg = 1;
    if (scene == 1) defocus_angle = 0.6;
    if (scene == 3) lookfrom[0] = 0.0, lookfrom[1] = 0.0, lookfrom[2] = 12.0;
    if (scene == 5) {  // mod.rs:301-313
        aspect_ratio = 1.0, vfov = 80.0;
        lookfrom[0] = 0.0, lookfrom[1] = 0.0, lookfrom[2] = 9.0;
    } else if (scene == 6) {  // mod.rs:342-354
        vfov = 20.0;
        lookfrom[0] = 26.0, lookfrom[1] = 3.0, lookfrom[2] = 6.0;
        lookat[1] = 2.0;
        background[0] = background[1] = background[2] = 0.0;
    } else if (scene == 7 || scene == 8 || scene == kBook3Scene) {  // mod.rs:412-423, 490-501; book 3 mod.rs:146-158
        aspect_ratio = 1.0, image_width = 600, samples_per_pixel = scene == kBook3Scene ? 100 : 200, vfov = 40.0;
        lookfrom[0] = 278.0, lookfrom[1] = 278.0, lookfrom[2] = -800.0;
        lookat[0] = 278.0, lookat[1] = 278.0, lookat[2] = 0.0;
        background[0] = background[1] = background[2] = 0.0;
    } else if (scene == 9 || scene == 10) {  // final_scene (mod.rs:570-585), main.rs:78-79 arguments
        aspect_ratio = 1.0, vfov = 40.0;
        image_width = scene == 9 ? 800 : 400;
        samples_per_pixel = scene == 9 ? 10000 : 250;
        max_depth = scene == 9 ? 40 : 4;
        lookfrom[0] = 478.0, lookfrom[1] = 278.0, lookfrom[2] = -600.0;
        lookat[0] = 278.0, lookat[1] = 278.0, lookat[2] = 0.0;
        background[0] = background[1] = background[2] = 0.0;
    }
    rrt_apply_overrides(ov, 2, &aspect_ratio, &image_width, &samples_per_pixel, &max_depth, &vfov, lookfrom, lookat,
                        vup, &defocus_angle, &focus_dist, background, &has_bg);

    SmallRng rng(seed);
    auto random_double = [&]() { return rng.gen_range_f64(0.0, 1.0); };
    auto random_range = [&](double lo, double hi) { return rng.gen_range_f64(lo, hi); };
    std::vector<RrtSphere> sph;
    std::vector<RrtMaterial> mat;
    std::vector<float> mot;
    std::vector<RrtPerlin> tables;
    std::vector<RrtQuad> qds, bqs;
    std::vector<RrtMedium> meds;
    std::vector<RrtLight> lights;
    uint32_t uses_texture0 = 0;
    auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
    auto add_material = [&](uint32_t kind, float r, float g, float b, float w, float ref_idx, uint32_t p0, uint32_t p1) {
        RrtMaterial m{};
        put4(m.albedo_fuzz, r, g, b, w);
        m.kind = kind;
        m.ref_idx = ref_idx;
        m._pad[0] = p0;
        m._pad[1] = p1;
        mat.push_back(m);
        return (uint32_t)(mat.size() - 1);
    };
    // CheckerTexture::from_colors(0.32, (.2,.3,.1), (.9,.9,.9)) (mod.rs:86-90): inv_scale = 1/scale
    auto checker = [&]() {
        return add_material(RRT_MAT_CHECKER_LAMBERTIAN, 0.2f, 0.3f, 0.1f, (float)(1.0 / 0.32), 0.9f, bits(0.9f),
                            bits(0.9f));
    };
    auto add_sphere = [&](D3 c, double r, uint32_t m, D3 move) {
        RrtSphere s{};
        put4(s.center_radius, (float)c.x, (float)c.y, (float)c.z, (float)r);
        s.material_index = m;
        sph.push_back(s);
        mot.insert(mot.end(), {(float)move.x, (float)move.y, (float)move.z, 0.0f});
    };
    const D3 still = d3(0.0, 0.0, 0.0);
    // Quad::new (quad.rs:21-37) under an optional RotateY(deg) then Translate(offset)
    // (hittable.rs:65-170), baked to world space in f64: a point p goes to
    // (cos x + sin z, y, -sin x + cos z) + offset, an edge vector rotates only.
    struct Xform {
        double c = 1.0, s = 0.0;
        D3 off = d3(0.0, 0.0, 0.0);
    };
    auto rot = [](const Xform &x, D3 a) { return d3(x.c * a.x + x.s * a.z, a.y, -x.s * a.x + x.c * a.z); };
    auto add_quad_to = [&](std::vector<RrtQuad> &dst, D3 q, D3 u, D3 v, uint32_t m, const Xform &x) {
        const D3 wq = rot(x, q) + x.off, wu = rot(x, u), wv = rot(x, v);
        RrtQuad r{};
        put4(r.q, (float)wq.x, (float)wq.y, (float)wq.z, 0.0f);
        put4(r.u, (float)wu.x, (float)wu.y, (float)wu.z, 0.0f);
        put4(r.v, (float)wv.x, (float)wv.y, (float)wv.z, 0.0f);
        r.material_index = m;
        dst.push_back(r);
    };
    auto add_quad = [&](D3 q, D3 u, D3 v, uint32_t m, const Xform &x) { add_quad_to(qds, q, u, v, m, x); };
    const Xform ident;
    // make_box (quad.rs:95-119): six faces into `dst` (the scene's quads, or a medium boundary)
    auto make_box_to = [&](std::vector<RrtQuad> &dst, D3 a, D3 b, uint32_t m, const Xform &x) {
        const D3 lo = d3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
        const D3 hi = d3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
        const D3 dx = d3(hi.x - lo.x, 0.0, 0.0), dy = d3(0.0, hi.y - lo.y, 0.0), dz = d3(0.0, 0.0, hi.z - lo.z);
        const D3 ndx = d3(-dx.x, 0.0, 0.0), ndz = d3(0.0, 0.0, -dz.z);
        add_quad_to(dst, d3(lo.x, lo.y, hi.z), dx, dy, m, x);
        add_quad_to(dst, d3(hi.x, lo.y, hi.z), ndz, dy, m, x);
        add_quad_to(dst, d3(hi.x, lo.y, lo.z), ndx, dy, m, x);
        add_quad_to(dst, d3(lo.x, lo.y, lo.z), dz, dy, m, x);
        add_quad_to(dst, d3(lo.x, hi.y, hi.z), dx, ndz, m, x);
        add_quad_to(dst, d3(lo.x, lo.y, lo.z), dx, dz, m, x);
    };
    auto make_box = [&](D3 a, D3 b, uint32_t m, const Xform &x) { make_box_to(qds, a, b, m, x); };
    // ConstantMedium::from_color (constant_medium.rs:30-36): Isotropic(albedo) phase function
    auto medium = [&](uint32_t kind, D3 c, double r, uint32_t first, uint32_t count, double density, D3 albedo) {
        RrtMedium md{};
        put4(md.sphere, (float)c.x, (float)c.y, (float)c.z, (float)r);
        md.boundary_kind = kind;
        md.first = first;
        md.count = count;
        md.material_index = add_material(RRT_MAT_ISOTROPIC, (float)albedo.x, (float)albedo.y, (float)albedo.z, 0.0f,
                                         1.0f, 0, 0);
        md.density = (float)density;
        meds.push_back(md);
    };
    auto box_medium = [&](D3 a, D3 b, const Xform &x, double density, D3 albedo) {
        const uint32_t first = (uint32_t)bqs.size();
        make_box_to(bqs, a, b, 0, x);
        medium(RRT_BOUNDARY_QUADS, d3(0, 0, 0), 0.0, first, 6, density, albedo);
    };
    auto rotate_translate = [](double deg, D3 off) {  // RotateY::new (hittable.rs:100-103)
        Xform x;
        const double rad = degrees_to_radians(deg);
        x.s = std::sin(rad);
        x.c = std::cos(rad);
        x.off = off;
        return x;
    };
    auto lambertian = [&](float r, float g, float b) { return add_material(RRT_MAT_LAMBERTIAN, r, g, b, 0.0f, 1.0f, 0, 0); };
    auto diffuse_light = [&](float e) { return add_material(RRT_MAT_DIFFUSE_LIGHT, e, e, e, 0.0f, 1.0f, 0, 0); };
    auto perlin_table = [&]() {  // Perlin::new (perlin.rs:12-22)
        RrtPerlin t{};
        for (int i = 0; i < 256; ++i) {
            double v[3];
            for (double &x : v) x = random_range(-1.0, 1.0);
            const D3 u = unit_vector(d3(v[0], v[1], v[2]));
            t.randvec[i][0] = (float)u.x;
            t.randvec[i][1] = (float)u.y;
            t.randvec[i][2] = (float)u.z;
        }
        for (uint16_t *perm : {t.perm_x, t.perm_y, t.perm_z}) {  // perlin_generate_perm / permute (perlin.rs:70-82)
            for (int i = 0; i < 256; ++i) perm[i] = (uint16_t)i;
            for (int i = 255; i > 0; --i) {
                const int target = (int)random_range(0.0, (double)(i + 1));
                std::swap(perm[i], perm[target]);
            }
        }
        tables.push_back(t);
        return (uint32_t)(tables.size() - 1);
    };
    if (scene == 1) {  // bouncing_spheres (mod.rs:83-135)
        add_sphere(d3(0.0, -1000.0, 0.0), 1000.0, checker(), still);
        for (int a = -11; a < 11; ++a) {
            for (int b = -11; b < 11; ++b) {
                const double choose_mat = random_double();
                const double cx = (double)a + 0.9 * random_double();
                const double cz = (double)b + 0.9 * random_double();
                const D3 center = d3(cx, 0.2, cz);
                if (length(center - d3(4.0, 0.2, 0.0)) > 0.9) {
                    if (choose_mat < 0.8) {
                        double c1[3], c2[3];  // Color::random() * Color::random()
                        for (double &v : c1) v = random_double();
                        for (double &v : c2) v = random_double();
                        const uint32_t m = add_material(RRT_MAT_LAMBERTIAN, (float)(c1[0] * c2[0]), (float)(c1[1] * c2[1]),
                                                        (float)(c1[2] * c2[2]), 0.0f, 1.0f, 0, 0);
                        const D3 center2 = center + d3(0.0, random_double() * 0.5, 0.0);
                        add_sphere(center, 0.2, m, center2 - center);  // Sphere::new_moving
                    } else if (choose_mat < 0.95) {
                        double al[3];
                        for (double &v : al) v = random_range(0.5, 1.0);
                        const double fuzz = random_double() * 0.5;
                        add_sphere(center, 0.2,
                                   add_material(RRT_MAT_METAL, (float)al[0], (float)al[1], (float)al[2], (float)fuzz,
                                                1.0f, 0, 0),
                                   still);
                    } else {
                        add_sphere(center, 0.2, add_material(RRT_MAT_DIELECTRIC, 1, 1, 1, 0, 1.5f, 0, 0), still);
                    }
                }
            }
        }
        add_sphere(d3(0.0, 1.0, 0.0), 1.0, add_material(RRT_MAT_DIELECTRIC, 1, 1, 1, 0, 1.5f, 0, 0), still);
        add_sphere(d3(-4.0, 1.0, 0.0), 1.0, add_material(RRT_MAT_LAMBERTIAN, 0.4f, 0.2f, 0.1f, 0, 1.0f, 0, 0), still);
        add_sphere(d3(4.0, 1.0, 0.0), 1.0, add_material(RRT_MAT_METAL, 0.7f, 0.6f, 0.5f, 0.0f, 1.0f, 0, 0), still);
    } else if (scene == 2) {  // checkered_spheres (mod.rs:157-175)
        add_sphere(d3(0.0, -10.0, 0.0), 10.0, checker(), still);
        add_sphere(d3(0.0, 10.0, 0.0), 10.0, checker(), still);
    } else if (scene == 3) {  // earth (mod.rs:196-201): the image is texture 0
        add_sphere(d3(0.0, 0.0, 0.0), 2.0, add_material(RRT_MAT_TEXTURED_LAMBERTIAN, 0, 0, 0, 0, 1.0f, 0, 0), still);
        uses_texture0 = 1;
    } else if (scene == 4 || scene == 6) {
        // perlin_spheres (mod.rs:222-235) / simple_light (mod.rs:318-340): one NoiseTexture(4)
        // shared by the ground and the sphere
        const uint32_t t = perlin_table();
        const uint32_t m = add_material(RRT_MAT_NOISE_LAMBERTIAN, 0.5f, 0.5f, 0.5f, 4.0f, 1.0f, t, 0);
        add_sphere(d3(0.0, -1000.0, 0.0), 1000.0, m, still);
        add_sphere(d3(0.0, 2.0, 0.0), 2.0, m, still);
        if (scene == 6) {
            const uint32_t light = diffuse_light(4.0f);
            add_sphere(d3(0.0, 7.0, 0.0), 2.0, light, still);
            add_quad(d3(3.0, 1.0, -2.0), d3(2.0, 0.0, 0.0), d3(0.0, 2.0, 0.0), light, ident);
        }
    } else if (scene == 5) {  // quads (mod.rs:257-299)
        add_quad(d3(-3, -2, 5), d3(0, 0, -4), d3(0, 4, 0), lambertian(1.0f, 0.2f, 0.2f), ident);
        add_quad(d3(-2, -2, 0), d3(4, 0, 0), d3(0, 4, 0), lambertian(0.2f, 1.0f, 0.2f), ident);
        add_quad(d3(3, -2, 1), d3(0, 0, 4), d3(0, 4, 0), lambertian(0.2f, 0.2f, 1.0f), ident);
        add_quad(d3(-2, 3, 1), d3(4, 0, 0), d3(0, 0, 4), lambertian(1.0f, 0.5f, 0.0f), ident);
        add_quad(d3(-2, -3, 5), d3(4, 0, 0), d3(0, 0, -4), lambertian(0.2f, 0.8f, 0.8f), ident);
    } else if (scene == 7) {  // cornell_box (mod.rs:359-410)
        const uint32_t red = lambertian(0.65f, 0.05f, 0.05f), white = lambertian(0.73f, 0.73f, 0.73f);
        const uint32_t green = lambertian(0.12f, 0.45f, 0.15f), light = diffuse_light(15.0f);
        add_quad(d3(555, 0, 0), d3(0, 555, 0), d3(0, 0, 555), green, ident);
        add_quad(d3(0, 0, 0), d3(0, 555, 0), d3(0, 0, 555), red, ident);
        add_quad(d3(343, 554, 332), d3(-130, 0, 0), d3(0, 0, -105), light, ident);
        add_quad(d3(0, 0, 0), d3(555, 0, 0), d3(0, 0, 555), white, ident);
        add_quad(d3(555, 555, 555), d3(-555, 0, 0), d3(0, 0, -555), white, ident);
        add_quad(d3(0, 0, 555), d3(555, 0, 0), d3(0, 555, 0), white, ident);
        make_box(d3(0, 0, 0), d3(165, 330, 165), white, rotate_translate(15.0, d3(265, 0, 295)));
        make_box(d3(0, 0, 0), d3(165, 165, 165), white, rotate_translate(-18.0, d3(130, 0, 65)));
    } else if (scene == 8) {  // cornell_smoke (mod.rs:432-488): the two boxes become media
        const uint32_t red = lambertian(0.65f, 0.05f, 0.05f), white = lambertian(0.73f, 0.73f, 0.73f);
        const uint32_t green = lambertian(0.12f, 0.45f, 0.15f), light = diffuse_light(7.0f);
        add_quad(d3(555, 0, 0), d3(0, 555, 0), d3(0, 0, 555), green, ident);
        add_quad(d3(0, 0, 0), d3(0, 555, 0), d3(0, 0, 555), red, ident);
        add_quad(d3(113, 554, 127), d3(330, 0, 0), d3(0, 0, 305), light, ident);
        add_quad(d3(0, 555, 0), d3(555, 0, 0), d3(0, 0, 555), white, ident);
        add_quad(d3(0, 0, 0), d3(555, 0, 0), d3(0, 0, 555), white, ident);
        add_quad(d3(0, 0, 555), d3(555, 0, 0), d3(0, 555, 0), white, ident);
        box_medium(d3(0, 0, 0), d3(165, 330, 165), rotate_translate(15.0, d3(265, 0, 295)), 0.01, d3(0, 0, 0));
        box_medium(d3(0, 0, 0), d3(165, 165, 165), rotate_translate(-18.0, d3(130, 0, 65)), 0.01, d3(1, 1, 1));
    } else if (scene == kBook3Scene) {  // the_rest_of_your_life/mod.rs:69-143
        const uint32_t red = lambertian(0.65f, 0.05f, 0.05f), white = lambertian(0.73f, 0.73f, 0.73f);
        const uint32_t green = lambertian(0.12f, 0.45f, 0.15f), light = diffuse_light(15.0f);
        add_quad(d3(555, 0, 0), d3(0, 0, 555), d3(0, 555, 0), green, ident);
        add_quad(d3(0, 0, 555), d3(0, 0, -555), d3(0, 555, 0), red, ident);
        add_quad(d3(0, 555, 0), d3(555, 0, 0), d3(0, 0, 555), white, ident);
        add_quad(d3(0, 0, 555), d3(555, 0, 0), d3(0, 0, -555), white, ident);
        add_quad(d3(555, 0, 555), d3(-555, 0, 0), d3(0, 555, 0), white, ident);
        add_quad(d3(213, 554, 227), d3(130, 0, 0), d3(0, 0, 105), light, ident);
        make_box(d3(0, 0, 0), d3(165, 330, 165), white, rotate_translate(15.0, d3(265, 0, 295)));
        add_sphere(d3(190, 90, 190), 90.0, add_material(RRT_MAT_DIELECTRIC, 1, 1, 1, 0, 1.5f, 0, 0), still);
        RrtLight lq{};  // lights: the light quad (reversed edges) and the glass sphere
        lq.kind = RRT_LIGHT_QUAD;
        put4(lq.a, 343.0f, 554.0f, 332.0f, 0.0f);
        put4(lq.u, -130.0f, 0.0f, 0.0f, 0.0f);
        put4(lq.v, 0.0f, 0.0f, -105.0f, 0.0f);
        lights.push_back(lq);
        RrtLight ls{};
        ls.kind = RRT_LIGHT_SPHERE;
        put4(ls.a, 190.0f, 90.0f, 190.0f, 90.0f);
        lights.push_back(ls);
    } else {  // final_scene (mod.rs:503-587)
        const uint32_t ground = lambertian(0.48f, 0.83f, 0.53f);
        for (int i = 0; i < 20; ++i)
            for (int j = 0; j < 20; ++j) {
                const double w = 100.0;
                const double x0 = -1000.0 + i * w, z0 = -1000.0 + j * w, y0 = 0.0;
                const double x1 = x0 + w, y1 = random_double() * 100.0 + 1.0, z1 = z0 + w;
                make_box(d3(x0, y0, z0), d3(x1, y1, z1), ground, ident);
            }
        add_quad(d3(123, 554, 147), d3(300, 0, 0), d3(0, 0, 265), diffuse_light(7.0f), ident);
        const D3 center1 = d3(400, 400, 200);
        add_sphere(center1, 50.0, lambertian(0.7f, 0.3f, 0.1f), d3(30, 0, 0));  // new_moving: center2 - center1
        add_sphere(d3(260, 150, 45), 50.0, add_material(RRT_MAT_DIELECTRIC, 1, 1, 1, 0, 1.5f, 0, 0), still);
        add_sphere(d3(0, 150, 145), 50.0, add_material(RRT_MAT_METAL, 0.8f, 0.8f, 0.9f, 1.0f, 1.0f, 0, 0), still);
        // boundary sphere: a dielectric surface and the boundary of a medium
        add_sphere(d3(360, 150, 145), 70.0, add_material(RRT_MAT_DIELECTRIC, 1, 1, 1, 0, 1.5f, 0, 0), still);
        medium(RRT_BOUNDARY_SPHERE, d3(360, 150, 145), 70.0, 0, 0, 0.2, d3(0.2, 0.4, 0.9));
        medium(RRT_BOUNDARY_SPHERE, d3(0, 0, 0), 5000.0, 0, 0, 0.0001, d3(1, 1, 1));  // boundary only
        add_sphere(d3(400, 200, 400), 100.0, add_material(RRT_MAT_TEXTURED_LAMBERTIAN, 0, 0, 0, 0, 1.0f, 0, 0), still);
        uses_texture0 = 1;
        const uint32_t t = perlin_table();  // NoiseTexture::new(0.2)
        add_sphere(d3(220, 280, 300), 80.0, add_material(RRT_MAT_NOISE_LAMBERTIAN, 0.5f, 0.5f, 0.5f, 0.2f, 1.0f, t, 0),
                   still);
        const uint32_t white = lambertian(0.73f, 0.73f, 0.73f);
        const Xform xf = rotate_translate(15.0, d3(-100, 270, 395));
        for (int k = 0; k < 1000; ++k) {  // Vec3::random_range(0, 165): x, y, z draws
            double c[3];
            for (double &v : c) v = random_range(0.0, 165.0);
            add_sphere(rot(xf, d3(c[0], c[1], c[2])) + xf.off, 10.0, white, still);
        }
    }
    const uint32_t sample_seed = rng.next_u32();
    if (scene == kBook3Scene) {  // Camera::initialize: sqrt_spp^2 stratified samples (camera.rs:115-117)
        const int32_t sq = (int32_t)std::sqrt((double)std::max(samples_per_pixel, 1));
        samples_per_pixel = sq * sq;
    }
    RrtBookScene &o = *out;
    o.n_spheres = (uint32_t)sph.size();
    o.n_materials = (uint32_t)mat.size();
    o.n_quads = (uint32_t)qds.size();
    o.n_perlin = (uint32_t)tables.size();
    o.n_media = (uint32_t)meds.size();
    o.n_boundary_quads = (uint32_t)bqs.size();
    o.n_lights = (uint32_t)lights.size();
    o.uses_texture0 = uses_texture0;
    o.flags = RRT_FLAG_RAY_TIME | (scene == kBook3Scene ? RRT_FLAG_BOOK3 : 0u);
    int rc = rrt_make_camera(aspect_ratio, image_width, samples_per_pixel, max_depth, vfov, lookfrom, lookat, vup,
                             defocus_angle, focus_dist, has_bg ? background : nullptr, sample_seed,
                             (uint32_t)sph.size(), &o.camera);
    if (rc) return rc;
    // copy out each array whose cap is set (cap 0 = sizing only)
    auto put = [&](auto *dst, uint32_t cap, const auto &src, const char *what) -> int32_t {
        if (cap == 0) return RRT_OK;
        if (cap < src.size() || !dst)
            return fail(RRT_E_INVALID, std::string(what) + "_cap too small (need " + std::to_string(src.size()) + ")");
        if (!src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(src[0]));
        return RRT_OK;
    };
    if ((rc = put(o.spheres, o.sphere_cap, sph, "sphere")) || (rc = put(o.materials, o.material_cap, mat, "material")) ||
        (rc = put(o.quads, o.quad_cap, qds, "quad")) || (rc = put(o.perlin, o.perlin_cap, tables, "perlin")) ||
        (rc = put(o.media, o.media_cap, meds, "media")) ||
        (rc = put(o.boundary_quads, o.boundary_quad_cap, bqs, "boundary_quad")) ||
        (rc = put(o.lights, o.light_cap, lights, "light")))
        return rc;
    if (o.sphere_motion && o.sphere_cap >= sph.size() && !mot.empty())
        std::memcpy(o.sphere_motion, mot.data(), mot.size() * sizeof(float));
    return RRT_OK;
}

int32_t rrt_build_next_week_scene(int32_t scene, const RrtOverrides *ov, uint64_t seed, RrtBookScene *out) {
    if (scene < 1 || scene > 10)
        return fail(RRT_E_INVALID, "book-2 scene must be 1 bouncing_spheres, 2 checkered_spheres, 3 earth, "
                                   "4 perlin_spheres, 5 quads, 6 simple_light, 7 cornell_box, 8 cornell_smoke, "
                                   "9 final_scene(800, 10000, 40), 10 final_scene(400, 250, 4)");
    return build_book_scene(scene, ov, seed, out);
}

int32_t rrt_build_rest_of_your_life_scene(const RrtOverrides *ov, uint64_t seed, RrtBookScene *out) {
    return build_book_scene(kBook3Scene, ov, seed, out);
}

}  // extern "C"

// ---- the object-graph flattener -------------------------------------------
namespace {

// RotateY then Translate as one affine map of the xz plane (hittable.rs:65-170): a point p goes
// to (c x + s z, y, -s x + c z) + off, a vector rotates only.
struct FXform {
    double c = 1.0, s = 0.0;
    D3 off = d3(0.0, 0.0, 0.0);
    D3 vec(D3 v) const { return d3(c * v.x + s * v.z, v.y, -s * v.x + c * v.z); }
    D3 point(D3 p) const { return vec(p) + off; }
};
// outer after inner
FXform compose(const FXform &outer, const FXform &inner) {
    FXform r;
    r.c = outer.c * inner.c - outer.s * inner.s;
    r.s = outer.s * inner.c + outer.c * inner.s;
    r.off = outer.vec(inner.off) + outer.off;
    return r;
}

struct Flattener {
    const RrtSceneNode *nodes;
    uint32_t n_nodes;
    const uint32_t *children;
    uint32_t n_children;
    std::vector<RrtSphere> sph;
    std::vector<float> mot;
    std::vector<RrtQuad> qds, bqs;
    std::vector<RrtMedium> meds;
    std::string err;

    bool walk(uint32_t id, const FXform &xf, int depth, bool in_medium) {
        if (depth > 64) return err = "object graph deeper than 64 (a cycle?)", false;
        if (id >= n_nodes) return err = "node index " + std::to_string(id) + " out of range", false;
        const RrtSceneNode &n = nodes[id];
        auto child = [&](uint32_t k) -> int64_t {
            if ((uint64_t)n.first + k >= n_children) return -1;
            return children[n.first + k];
        };
        switch (n.kind) {
            case RRT_NODE_SPHERE: {
                const D3 c = xf.point(d3(n.a[0], n.a[1], n.a[2]));
                const D3 m = xf.vec(d3(n.b[0], n.b[1], n.b[2]));
                RrtSphere sp{};
                put4(sp.center_radius, (float)c.x, (float)c.y, (float)c.z, (float)n.a[3]);
                sp.material_index = n.material;
                sph.push_back(sp);
                mot.insert(mot.end(), {(float)m.x, (float)m.y, (float)m.z, 0.0f});
                return true;
            }
            case RRT_NODE_QUAD: {
                const D3 q = xf.point(d3(n.a[0], n.a[1], n.a[2]));
                const D3 u = xf.vec(d3(n.b[0], n.b[1], n.b[2])), v = xf.vec(d3(n.c[0], n.c[1], n.c[2]));
                RrtQuad r{};
                put4(r.q, (float)q.x, (float)q.y, (float)q.z, 0.0f);
                put4(r.u, (float)u.x, (float)u.y, (float)u.z, 0.0f);
                put4(r.v, (float)v.x, (float)v.y, (float)v.z, 0.0f);
                r.material_index = n.material;
                qds.push_back(r);
                return true;
            }
            case RRT_NODE_LIST:
            case RRT_NODE_BVH:
                for (uint32_t k = 0; k < n.count; ++k) {
                    const int64_t c = child(k);
                    if (c < 0) return err = "node " + std::to_string(id) + ": children out of range", false;
                    if (!walk((uint32_t)c, xf, depth + 1, in_medium)) return false;
                }
                return true;
            case RRT_NODE_TRANSLATE:
            case RRT_NODE_ROTATE_Y: {
                const int64_t c = n.count == 1 ? child(0) : -1;
                if (c < 0) return err = "node " + std::to_string(id) + ": a transform takes one child", false;
                FXform t;
                if (n.kind == RRT_NODE_TRANSLATE) {
                    t.off = d3(n.a[0], n.a[1], n.a[2]);
                } else {  // RotateY::new (hittable.rs:100-103)
                    const double rad = degrees_to_radians(n.a[0]);
                    t.s = std::sin(rad);
                    t.c = std::cos(rad);
                }
                return walk((uint32_t)c, compose(xf, t), depth + 1, in_medium);
            }
            case RRT_NODE_CONSTANT_MEDIUM: {
                if (in_medium) return err = "node " + std::to_string(id) + ": a medium inside a medium boundary", false;
                const int64_t c = n.count == 1 ? child(0) : -1;
                if (c < 0) return err = "node " + std::to_string(id) + ": a medium takes one boundary child", false;
                Flattener sub{nodes, n_nodes, children, n_children, {}, {}, {}, {}, {}, {}};
                if (!sub.walk((uint32_t)c, xf, depth + 1, true)) return err = sub.err, false;
                RrtMedium md{};
                md.material_index = n.material;
                md.density = (float)n.a[0];
                if (sub.sph.size() == 1 && sub.qds.empty()) {
                    if (sub.mot[0] != 0.0f || sub.mot[1] != 0.0f || sub.mot[2] != 0.0f)
                        return err = "node " + std::to_string(id) + ": moving medium boundaries are not supported", false;
                    md.boundary_kind = RRT_BOUNDARY_SPHERE;
                    std::memcpy(md.sphere, sub.sph[0].center_radius, sizeof(md.sphere));
                } else if (sub.sph.empty() && !sub.qds.empty()) {
                    md.boundary_kind = RRT_BOUNDARY_QUADS;
                    md.first = (uint32_t)bqs.size();
                    md.count = (uint32_t)sub.qds.size();
                    bqs.insert(bqs.end(), sub.qds.begin(), sub.qds.end());
                } else {
                    return err = "node " + std::to_string(id) + ": a medium boundary is one sphere or quads only", false;
                }
                meds.push_back(md);
                return true;
            }
            default:
                return err = "node " + std::to_string(id) + ": unknown kind", false;
        }
    }
};

}  // namespace

extern "C" {

int32_t rrt_flatten_scene(const RrtSceneNode *nodes, uint32_t n_nodes, const uint32_t *children, uint32_t n_children,
                          uint32_t root, RrtBookScene *out) {
    if (!out || (n_nodes && !nodes) || (n_children && !children)) return fail(RRT_E_INVALID, "null argument");
    Flattener f{nodes, n_nodes, children, n_children, {}, {}, {}, {}, {}, {}};
    if (!f.walk(root, FXform{}, 0, false)) return fail(RRT_E_INVALID, "rrt_flatten_scene: " + f.err);
    RrtBookScene &o = *out;
    o.n_spheres = (uint32_t)f.sph.size();
    o.n_quads = (uint32_t)f.qds.size();
    o.n_media = (uint32_t)f.meds.size();
    o.n_boundary_quads = (uint32_t)f.bqs.size();
    auto put = [&](auto *dst, uint32_t cap, const auto &src, const char *what) -> int32_t {
        if (cap == 0) return RRT_OK;
        if (cap < src.size() || !dst)
            return fail(RRT_E_INVALID, std::string(what) + "_cap too small (need " + std::to_string(src.size()) + ")");
        if (!src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(src[0]));
        return RRT_OK;
    };
    int32_t rc;
    if ((rc = put(o.spheres, o.sphere_cap, f.sph, "sphere")) || (rc = put(o.quads, o.quad_cap, f.qds, "quad")) ||
        (rc = put(o.media, o.media_cap, f.meds, "media")) ||
        (rc = put(o.boundary_quads, o.boundary_quad_cap, f.bqs, "boundary_quad")))
        return rc;
    if (o.sphere_motion && o.sphere_cap >= f.sph.size() && !f.mot.empty())
        std::memcpy(o.sphere_motion, f.mot.data(), f.mot.size() * sizeof(float));
    return RRT_OK;
}

// ---- render_io.rs:3-31 -------------------------------------------------------------------
static inline uint8_t quantize_channel(float x, float scale) {
    float r = x * scale;
    if (!std::isfinite(r)) r = 0.0f;
    r = std::sqrt(r < 0.0f ? 0.0f : r);
    if (r < 0.0f) r = 0.0f;  // f32::clamp(0.0, 0.999)
    if (r > 0.999f) r = 0.999f;
    return (uint8_t)(int)(r * 256.0f);
}

}  // extern "C"

// Host threads for the output step: RRT_HOST_THREADS, else OMP_NUM_THREADS, else the
// hardware count; at most 16 (the GPU box's CPU share per GPU).
static unsigned host_threads() {
    const char *e = std::getenv("RRT_HOST_THREADS");
    if (!e) e = std::getenv("OMP_NUM_THREADS");
    unsigned n = e ? (unsigned)std::max(1, std::atoi(e)) : std::max(1u, std::thread::hardware_concurrency());
    return std::min(n, 16u);
}

// fn(begin, end) over [0, n) in contiguous chunks, one per host thread (inline when small).
static void parallel_chunks(size_t n, size_t min_chunk, const std::function<void(size_t, size_t, unsigned)> &fn,
                            unsigned *n_chunks_out = nullptr) {
    const unsigned t = (unsigned)std::max<size_t>(1, std::min<size_t>(host_threads(), n / std::max<size_t>(min_chunk, 1)));
    if (n_chunks_out) *n_chunks_out = t;
    if (t <= 1) {
        fn(0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned i = 0; i < t; ++i) th.emplace_back(fn, n * i / t, n * (i + 1) / t, i);
    for (auto &x : th) x.join();
}

static void quantize_rgb8(size_t n_px, const float *accum, uint32_t spp, uint8_t *rgb8) {
    const float scale = spp > 0 ? 1.0f / (float)spp : 0.0f;
    parallel_chunks(n_px, 1u << 16, [&](size_t b, size_t e, unsigned) {
        for (size_t i = b; i < e; ++i)
            for (int c = 0; c < 3; ++c) rgb8[i * 3 + c] = quantize_channel(accum[i * 4 + c], scale);
    });
}

// color.rs:6-32 write_color for one channel of pixel_samples_scale * pixel_color (f64, the books
// CPU path's quantiser): linear_to_gamma (sqrt of a positive value, else 0), Interval(0, 0.999)
// clamp (NaN passes through: both comparisons are false), 256 * x `as i32` (NaN -> 0, +inf was
// clamped to 0.999 -> 255).
static inline uint8_t books_channel(double x) {
    x = x > 0.0 ? std::sqrt(x) : 0.0;
    if (x < 0.0) x = 0.0;
    if (x > 0.999) x = 0.999;
    const double v = 256.0 * x;
    return v != v ? (uint8_t)0 : (uint8_t)(int32_t)v;
}

template <class T>
static void quantize_rgb8_books(size_t n_px, const T *accum, uint32_t spp, uint8_t *rgb8) {
    const double scale = 1.0 / (double)spp;  // camera.rs:107 pixel_samples_scale (spp >= 1)
    parallel_chunks(n_px, 1u << 16, [&](size_t b, size_t e, unsigned) {
        for (size_t i = b; i < e; ++i)
            for (int c = 0; c < 3; ++c) rgb8[i * 3 + c] = books_channel(scale * (double)accum[i * 4 + c]);
    });
}

// Decimal strings of 0..255 (no leading zeros) for the P3 "r g b\n" lines.
struct DecTable {
    char s[256][4];
    uint8_t n[256];
    DecTable() {
        for (int v = 0; v < 256; ++v) n[v] = (uint8_t)std::snprintf(s[v], sizeof(s[v]), "%d", v);
    }
};
static const DecTable &dec_table() {
    static const DecTable t;
    return t;
}

// P3 / P6 bytes of an rgb8 image. P3 lines are "%u %u %u\n" per pixel (render_io.rs:27),
// formatted in parallel chunks at offsets from a prefix sum of the chunks' lengths.
static std::vector<char> format_pnm(uint32_t width, uint32_t height, const uint8_t *rgb8, bool binary) {
    const std::string head =
        std::string(binary ? "P6\n" : "P3\n") + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
    const size_t n_px = (size_t)width * height;
    std::vector<char> out;
    if (binary) {
        out.resize(head.size() + n_px * 3);
        std::memcpy(out.data(), head.data(), head.size());
        if (n_px) std::memcpy(out.data() + head.size(), rgb8, n_px * 3);
        return out;
    }
    const DecTable &T = dec_table();
    std::vector<size_t> len(host_threads() + 1, 0);
    unsigned chunks = 1;
    parallel_chunks(
        n_px, 1u << 16,
        [&](size_t b, size_t e, unsigned i) {
            size_t l = 0;
            for (size_t p = b; p < e; ++p) l += (size_t)T.n[rgb8[3 * p]] + T.n[rgb8[3 * p + 1]] + T.n[rgb8[3 * p + 2]] + 3;
            len[i + 1] = l;
        },
        &chunks);
    for (unsigned i = 0; i < chunks; ++i) len[i + 1] += len[i];
    out.resize(head.size() + len[chunks]);
    std::memcpy(out.data(), head.data(), head.size());
    parallel_chunks(n_px, 1u << 16, [&](size_t b, size_t e, unsigned i) {
        char *d = out.data() + head.size() + len[i];
        for (size_t p = b; p < e; ++p) {
            for (int c = 0; c < 3; ++c) {
                const uint8_t v = rgb8[3 * p + c];
                const char *sv = T.s[v];
                d[0] = sv[0];  // exactly the digits: chunks are written concurrently, no overrun
                if (T.n[v] > 1) d[1] = sv[1];
                if (T.n[v] > 2) d[2] = sv[2];
                d += T.n[v];
                *d++ = c < 2 ? ' ' : '\n';
            }
        }
    });
    return out;
}

static int32_t write_bytes(const std::vector<char> &buf, const char *path) {
    FILE *f = (!path || std::strcmp(path, "-") == 0) ? stdout : std::fopen(path, "wb");
    if (!f) return fail(RRT_E_IO, std::string("cannot open ") + path);
    const size_t w = std::fwrite(buf.data(), 1, buf.size(), f);
    if (f == stdout) std::fflush(f);
    else std::fclose(f);
    if (w != buf.size()) return fail(RRT_E_IO, "short write");
    return RRT_OK;
}

static int32_t copy_out(const std::vector<char> &bytes, char *buf, size_t cap, size_t *written) {
    *written = bytes.size();
    if (cap == 0) return RRT_OK;
    if (!buf || cap < bytes.size()) return fail(RRT_E_INVALID, "buffer too small");
    std::memcpy(buf, bytes.data(), bytes.size());
    return RRT_OK;
}

extern "C" {

int32_t rrt_quantize_accum(uint32_t width, uint32_t height, const float *accum, uint32_t spp, uint8_t *rgb8) {
    if ((!accum || !rgb8) && (size_t)width * height) return fail(RRT_E_INVALID, "null accum or rgb8");
    quantize_rgb8((size_t)width * height, accum, spp, rgb8);
    return RRT_OK;
}

int32_t rrt_quantize_accum_books(uint32_t width, uint32_t height, const float *accum, uint32_t spp, uint8_t *rgb8) {
    if ((!accum || !rgb8) && (size_t)width * height) return fail(RRT_E_INVALID, "null accum or rgb8");
    if (spp == 0) return fail(RRT_E_INVALID, "samples_per_pixel must be >= 1 (camera.rs pixel_samples_scale)");
    quantize_rgb8_books((size_t)width * height, accum, spp, rgb8);
    return RRT_OK;
}

int32_t rrt_quantize_accum_books_f64(uint32_t width, uint32_t height, const double *accum, uint32_t spp,
                                     uint8_t *rgb8) {
    if ((!accum || !rgb8) && (size_t)width * height) return fail(RRT_E_INVALID, "null accum or rgb8");
    if (spp == 0) return fail(RRT_E_INVALID, "samples_per_pixel must be >= 1 (camera.rs pixel_samples_scale)");
    quantize_rgb8_books((size_t)width * height, accum, spp, rgb8);
    return RRT_OK;
}

int32_t rrt_format_ppm_from_accum(uint32_t width, uint32_t height, const float *accum, uint32_t spp, char *buf,
                                  size_t cap, size_t *written) {
    if (!written) return fail(RRT_E_INVALID, "null written");
    if (!accum && (size_t)width * height) return fail(RRT_E_INVALID, "null accum");
    std::vector<uint8_t> rgb8((size_t)width * height * 3);
    quantize_rgb8((size_t)width * height, accum, spp, rgb8.data());
    return copy_out(format_pnm(width, height, rgb8.data(), false), buf, cap, written);
}

int32_t rrt_write_ppm_from_accum(uint32_t width, uint32_t height, const float *accum, uint32_t spp, const char *path) {
    if (!accum && (size_t)width * height) return fail(RRT_E_INVALID, "null accum");
    std::vector<uint8_t> rgb8((size_t)width * height * 3);
    quantize_rgb8((size_t)width * height, accum, spp, rgb8.data());
    return write_bytes(format_pnm(width, height, rgb8.data(), false), path);
}

int32_t rrt_format_pnm_from_rgb8(uint32_t width, uint32_t height, const uint8_t *rgb8, int32_t binary, char *buf,
                                 size_t cap, size_t *written) {
    if (!written) return fail(RRT_E_INVALID, "null written");
    if (!rgb8 && (size_t)width * height) return fail(RRT_E_INVALID, "null rgb8");
    return copy_out(format_pnm(width, height, rgb8, binary != 0), buf, cap, written);
}

int32_t rrt_write_pnm_from_rgb8(uint32_t width, uint32_t height, const uint8_t *rgb8, int32_t binary, const char *path) {
    if (!rgb8 && (size_t)width * height) return fail(RRT_E_INVALID, "null rgb8");
    return write_bytes(format_pnm(width, height, rgb8, binary != 0), path);
}

}  // extern "C"
