// test_graph_layout.cpp — tests of the C++ GraphLayout mirror
// (whisper-git_amd/host/graph_layout.hpp), written the way the reference's
// own tests are (/root/reference/src/commit_graph.rs:1585-1763), plus parity
// against the CPU oracle (oracle/wg_oracle.c — test infrastructure, the
// checker only) on generated DAGs.  Every computation under test runs in the
// HIP engine behind the C ABI.
//
//   test_graph_layout                 run every test (needs a gfx950 GPU)
//   test_graph_layout --list          list the tests
//   test_graph_layout NAME...         run the named tests
//   test_graph_layout --no-device     CPU box: GraphLayout must refuse (no fallback)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "graph_layout.hpp"
#include "wg_oracle.h"
#include "wg_synth.h"

using namespace wgraph;

namespace {

struct Failure {
    std::string what;
};

#define CHECK(cond)                                                                                   \
    do {                                                                                              \
        if (!(cond)) throw Failure{std::string(__FILE__ ":") + std::to_string(__LINE__) + ": " #cond}; \
    } while (0)
#define CHECK_EQ(a, b)                                                                                     \
    do {                                                                                                   \
        const auto va_ = (a);                                                                              \
        const auto vb_ = (b);                                                                              \
        if (!(va_ == vb_))                                                                                 \
            throw Failure{std::string(__FILE__ ":") + std::to_string(__LINE__) + ": " #a " == " #b " (" + \
                          std::to_string(va_) + " vs " + std::to_string(vb_) + ")"};                       \
    } while (0)

std::vector<std::pair<std::string, std::function<void()>>> &registry() {
    static std::vector<std::pair<std::string, std::function<void()>>> r;
    return r;
}
struct Reg {
    Reg(const char *name, std::function<void()> f) { registry().emplace_back(name, std::move(f)); }
};
#define TEST(name)                     \
    static void name();                \
    static Reg reg_##name(#name, name); \
    static void name()

// ---------------------------------------------------------------------------
// helpers: the reference's test_commit() and small hand-made lists
// ---------------------------------------------------------------------------
CommitInfo test_commit() { return CommitInfo{}; }   // :1744-1762

Oid oid_of(int k) {
    Oid o;
    o.bytes[0] = 0xC0;
    for (int i = 0; i < 4; i++) o.bytes[16 + i] = (uint8_t)(k >> (8 * i));
    return o;
}

// rows named 0..n-1, 60 s apart (all heights ROW_HEIGHT: uniform_offsets, :1627-1629)
std::vector<CommitInfo> uniform_list(int n) {
    std::vector<CommitInfo> v(n);
    for (int i = 0; i < n; i++) {
        v[i].id = oid_of(i);
        v[i].time = 1'000'000 - 60 * i;
    }
    return v;
}

// one colour's share of a row (the entries one edge contributes when its
// child is the only row of that colour)
RowGeometry of_color(const RowGeometry &r, Color c) {
    RowGeometry o;
    o.height = r.height;
    o.node_y = r.node_y;
    for (auto &v : r.full_verticals) if (v.second == c) o.full_verticals.push_back(v);
    for (auto &v : r.top_half_verticals) if (v.second == c) o.top_half_verticals.push_back(v);
    for (auto &v : r.bottom_half_verticals) if (v.second == c) o.bottom_half_verticals.push_back(v);
    for (auto &s : r.curves) if (s.color == c) o.curves.push_back(s);
    return o;
}

// A list whose only orphan-coloured edge is cross-lane, child at row 3
// (lane 1) and parent at row 3 + span - 1 (lane 0):
//   row 0  A -> G      lane 0 waits for G
//   row 1  B -> c      lane 1 waits for c
//   row 2  G           lane 0, frees slot 0
//   row 3  c (orphan) -> [outside, P]   lane 1; first parent outside the
//          list frees slot 1, the secondary P takes the lowest free slot, 0
//   rows   fillers, then P on lane 0
std::vector<CommitInfo> cross_lane_list(int span) {
    std::vector<CommitInfo> v = uniform_list(3 + span);
    const int P = 3 + span - 1;
    v[0].parent_ids = {oid_of(2)};
    v[1].parent_ids = {oid_of(3)};
    v[3].is_orphaned = true;
    v[3].parent_ids = {oid_of(1 << 20), oid_of(P)};
    return v;
}

}  // namespace

// ---------------------------------------------------------------------------
// The reference's known-answer tests (commit_graph.rs:1593-1742), at the
// GraphLayout boundary
// ---------------------------------------------------------------------------

// :1704-1723
TEST(compute_row_heights_clamps_to_min_for_dense_commits) {
    CommitInfo a = test_commit(), b = test_commit();
    a.time = 1'000'000;
    b.time = 1'000'000 - 60;
    const std::vector<float> h = compute_row_heights({a, b});
    CHECK_EQ(h.size(), (size_t)2);
    CHECK(std::fabs(h[0] - ROW_HEIGHT) < 1.0f);
    // Last row always uses minimum.
    CHECK(std::fabs(h[1] - ROW_HEIGHT) < 1.0f);
}

// :1725-1742
TEST(compute_row_heights_saturates_at_max_for_long_gaps) {
    CommitInfo a = test_commit(), b = test_commit();
    a.time = 1'000'000'000;
    b.time = 1'000'000'000 - 60 * 24 * 3600;
    const std::vector<float> h = compute_row_heights({a, b});
    const float expected = std::round(ROW_HEIGHT + MAX_EXTRA_HEIGHT);
    CHECK(std::fabs(h[0] - expected) < 1.0f);
}

// :1631-1653 — edge child_row 0 -> parent_row 3, same lane
TEST(decompose_same_lane_emits_top_full_bottom_verticals) {
    std::vector<CommitInfo> commits = uniform_list(4);
    commits[0].parent_ids = {oid_of(3)};   // rows 1, 2: parentless commits on lane 1
    GraphLayout layout;
    layout.build(commits);
    CHECK_EQ(layout.edges.size(), (size_t)1);
    CHECK_EQ(layout.edges[0].child_lane, layout.edges[0].parent_lane);
    const auto &rows = layout.row_geometry;
    // child row gets bottom-half (line emerges below the node).
    CHECK_EQ(rows[0].bottom_half_verticals.size(), (size_t)1);
    CHECK_EQ(rows[0].full_verticals.size(), (size_t)0);
    CHECK_EQ(rows[0].top_half_verticals.size(), (size_t)0);
    // intermediate rows get full verticals.
    CHECK_EQ(rows[1].full_verticals.size(), (size_t)1);
    CHECK_EQ(rows[2].full_verticals.size(), (size_t)1);
    // parent row gets top-half (line ends at the node).
    CHECK_EQ(rows[3].top_half_verticals.size(), (size_t)1);
}

// :1655-1679 — 4 spanned rows = 4 curve segments; no verticals on cross-lane
TEST(decompose_cross_lane_emits_one_curve_per_spanned_row) {
    const std::vector<CommitInfo> commits = cross_lane_list(4);
    GraphLayout layout;
    layout.build(commits);
    const CommitLayout *c = layout.get(oid_of(3));
    const CommitLayout *p = layout.get(oid_of(6));
    CHECK(c && p);
    CHECK(c->color == ORPHAN_COLOR);
    CHECK_EQ(c->lane, (size_t)1);
    CHECK_EQ(p->lane, (size_t)0);
    for (int r = 3; r <= 6; r++) {
        const RowGeometry g = of_color(layout.row_geometry[r], ORPHAN_COLOR);
        CHECK_EQ(g.curves.size(), (size_t)1);
        CHECK(g.full_verticals.empty());
        CHECK(g.top_half_verticals.empty());
        CHECK(g.bottom_half_verticals.empty());
    }
    for (int r = 0; r < 3; r++) CHECK(of_color(layout.row_geometry[r], ORPHAN_COLOR).curves.empty());
}

// :1681-1702 — child strip starts at NODE_Y, parent strip ends at NODE_Y
TEST(decompose_cross_lane_segment_y_spans_row_strip) {
    const std::vector<CommitInfo> commits = cross_lane_list(3);
    GraphLayout layout;
    layout.build(commits);
    const auto seg = [&](int r) { return of_color(layout.row_geometry[r], ORPHAN_COLOR).curves.at(0); };
    const CurveSegment row0 = seg(3), row1 = seg(4), row2 = seg(5);
    CHECK(std::fabs(row0.p0.second - NODE_Y) < 0.5f);
    CHECK(std::fabs(row0.p3.second - ROW_HEIGHT) < 0.5f);
    CHECK(std::fabs(row1.p0.second - 0.0f) < 0.5f);
    CHECK(std::fabs(row1.p3.second - ROW_HEIGHT) < 0.5f);
    CHECK(std::fabs(row2.p0.second - 0.0f) < 0.5f);
    CHECK(std::fabs(row2.p3.second - NODE_Y) < 0.5f);
}

// :1593-1607 (Cubic::t_at_y recovers the end points): the child row's
// segment starts at t = 0, the parent row's ends at t = 1, and the edge's
// middle row (y symmetric about the span's centre) passes x = midpoint
TEST(cubic_t_at_y_recovers_endpoints) {
    const std::vector<CommitInfo> commits = cross_lane_list(3);
    GraphLayout layout;
    layout.build(commits);
    const auto seg = [&](int r) { return of_color(layout.row_geometry[r], ORPHAN_COLOR).curves.at(0); };
    CHECK(std::fabs(seg(3).p0.first - 1.0f) < 1e-3f);     // child lane
    CHECK(std::fabs(seg(3).p0.second - NODE_Y) < 1e-3f);
    CHECK(std::fabs(seg(5).p3.first - 0.0f) < 1e-3f);     // parent lane
    CHECK(std::fabs(seg(5).p3.second - NODE_Y) < 1e-3f);
}

// :1609-1625 (subcurve end points match y_at): consecutive rows' segments
// meet — row r's end is row r+1's start in absolute y
TEST(cubic_subcurve_endpoints_match_y_at) {
    const std::vector<CommitInfo> commits = cross_lane_list(5);
    GraphLayout layout;
    layout.build(commits);
    for (int r = 3; r < 7; r++) {
        const CurveSegment a = of_color(layout.row_geometry[r], ORPHAN_COLOR).curves.at(0);
        const CurveSegment b = of_color(layout.row_geometry[r + 1], ORPHAN_COLOR).curves.at(0);
        CHECK(std::fabs(a.p3.second - layout.row_geometry[r].height - b.p0.second) < 1e-3f);
        CHECK(std::fabs(a.p3.first - b.p0.first) < 1e-3f);
    }
}

// ---------------------------------------------------------------------------
// GraphLayout semantics the reference's code defines (no reference test)
// ---------------------------------------------------------------------------

// :261-271, :353-354 — an empty list; build() resets the previous state
TEST(empty_list_and_rebuild_reset) {
    GraphLayout layout;
    layout.build(cross_lane_list(4));
    CHECK(layout.max_lane >= 1 && !layout.edges.empty());
    layout.build({});
    CHECK_EQ(layout.max_lane, (size_t)0);
    CHECK(layout.edges.empty() && layout.row_geometry.empty());
    CHECK_EQ(layout.graph_width, LANE_W);
    CHECK(layout.get(oid_of(3)) == nullptr);
}

// :273-274, :357 — duplicate ids: get() answers with the last row's layout
TEST(get_returns_the_last_occurrence) {
    std::vector<CommitInfo> commits = uniform_list(4);
    commits[0].parent_ids = {oid_of(9)};      // outside the list: lane 0 freed
    commits[1].parent_ids = {oid_of(3)};
    commits[2].id = oid_of(1);                // duplicate of row 1's id
    GraphLayout layout;
    layout.build(commits);
    const wgo_layout ref = [&] {
        CommitSoA soa(commits);
        wg_commits in = soa.view();
        wgo_layout L;
        CHECK_EQ(wgo_layout_build(&in, &L), 0);
        return L;
    }();
    for (size_t r = 0; r < commits.size(); r++) {
        const CommitLayout *l = layout.get(commits[r].id);
        CHECK(l != nullptr);
        CHECK_EQ(l->lane, (size_t)ref.lane[r]);
        CHECK(l->color == Color{ref.color[r]});
    }
    CHECK(layout.get(oid_of(9)) == nullptr);
    wgo_layout L = ref;
    wgo_layout_free(&L);
}

// :375, :386 — band_heights shorter than the list: missing bands are zero
TEST(row_geometry_with_short_band_list) {
    std::vector<CommitInfo> commits = cross_lane_list(4);
    GraphLayout layout;
    layout.build(commits);
    const auto g = layout.row_geometry_with_bands(commits, {PILLS_BAND_HEIGHT, 0.0f, PILLS_BAND_HEIGHT});
    CHECK_EQ(g.size(), commits.size());
    CHECK_EQ(g[0].height, ROW_HEIGHT + PILLS_BAND_HEIGHT);
    CHECK_EQ(g[0].node_y, NODE_Y + PILLS_BAND_HEIGHT);
    CHECK_EQ(g[2].node_y, NODE_Y + PILLS_BAND_HEIGHT);
    CHECK_EQ(g[3].node_y, NODE_Y);
    CHECK_EQ(g[6].height, ROW_HEIGHT);
    // the build's geometry (zero bands) is not touched by a frame's call
    CHECK_EQ(layout.row_geometry[0].node_y, NODE_Y);
    // an empty band list: every band is zero, the build's geometry again
    const auto g0 = layout.row_geometry_with_bands(commits, {});
    CHECK_EQ(g0.size(), commits.size());
    for (size_t r = 0; r < g0.size(); r++) {
        CHECK_EQ(g0[r].height, layout.row_geometry[r].height);
        CHECK_EQ(g0[r].node_y, NODE_Y);
        CHECK_EQ(g0[r].curves.size(), layout.row_geometry[r].curves.size());
    }
    // :372 — heights come from the list passed in: the same rows with a month
    // between two commits give that gap's height, as a layout built on it does
    std::vector<CommitInfo> gap = commits;
    for (size_t r = 2; r < gap.size(); r++) gap[r].time -= 30 * 86400;
    GraphLayout other;
    other.build(gap);
    const auto gg = layout.row_geometry_with_bands(gap, {});
    CHECK_EQ(gg.size(), other.row_geometry.size());
    bool differs = false;
    for (size_t r = 0; r < gg.size(); r++) {
        CHECK_EQ(gg[r].height, other.row_geometry[r].height);
        CHECK_EQ(gg[r].node_y, other.row_geometry[r].node_y);
        differs |= gg[r].height != layout.row_geometry[r].height;
    }
    CHECK(differs);
    // the next call without the gap is back on the build's heights
    const auto g1 = layout.row_geometry_with_bands(commits, {});
    for (size_t r = 0; r < g1.size(); r++) CHECK_EQ(g1[r].height, layout.row_geometry[r].height);
    // a list of another length: the edges index the built rows, refused
    bool threw = false;
    try {
        (void)layout.row_geometry_with_bands(uniform_list(3), {});
    } catch (const wgraph::Error &) {
        threw = true;
    }
    CHECK(threw);
}

// ---------------------------------------------------------------------------
// Parity against the CPU oracle on generated DAGs (SURVEY §8(d) presets)
// ---------------------------------------------------------------------------
namespace {

std::vector<CommitInfo> synth_list(int kind, uint64_t n, uint64_t seed, std::vector<float> *band) {
    wgs_params p;
    CHECK_EQ(wgs_preset(kind, n, seed, &p), 0);
    wgs_dag *d = wgs_generate(&p);
    CHECK(d != nullptr);
    uint64_t N, E;
    wgs_sizes(d, &N, &E);
    std::vector<uint8_t> oid(N * 20), poid(E * 20 + 20), flags(N);
    std::vector<int64_t> time(N);
    std::vector<uint32_t> poff(N + 1);
    band->assign(N, 0.0f);
    wgs_copy(d, oid.data(), time.data(), poff.data(), poid.data(), flags.data(), band->data());
    wgs_free(d);
    std::vector<CommitInfo> v(N);
    for (uint64_t i = 0; i < N; i++) {
        std::memcpy(v[i].id.bytes.data(), &oid[20 * i], 20);
        v[i].time = time[i];
        v[i].is_orphaned = flags[i] & WG_FLAG_ORPHAN;
        v[i].is_synthetic = flags[i] & WG_FLAG_SYNTHETIC;
        for (uint32_t k = poff[i]; k < poff[i + 1]; k++) {
            Oid o;
            std::memcpy(o.bytes.data(), &poid[20 * k], 20);
            v[i].parent_ids.push_back(o);
        }
    }
    return v;
}

void same_geometry(const std::vector<RowGeometry> &g, const wgo_geometry &o) {
    CHECK_EQ(g.size(), (size_t)o.n);
    for (size_t r = 0; r < g.size(); r++) {
        CHECK_EQ(std::memcmp(&g[r].height, &o.height[r], 4), 0);   // bit-exact f32
        CHECK_EQ(std::memcmp(&g[r].node_y, &o.node_y[r], 4), 0);
        std::vector<uint32_t> vert;
        for (auto &v : g[r].full_verticals) vert.push_back((uint32_t)v.first | WG_VERT_FULL << 24 | (uint32_t)v.second.index << 28);
        for (auto &v : g[r].top_half_verticals) vert.push_back((uint32_t)v.first | WG_VERT_TOP << 24 | (uint32_t)v.second.index << 28);
        for (auto &v : g[r].bottom_half_verticals)
            vert.push_back((uint32_t)v.first | WG_VERT_BOTTOM << 24 | (uint32_t)v.second.index << 28);
        CHECK_EQ(vert.size(), (size_t)(o.vert_off[r + 1] - o.vert_off[r]));
        CHECK(vert.empty() || std::memcmp(vert.data(), o.vert + o.vert_off[r], vert.size() * 4) == 0);
        CHECK_EQ(g[r].curves.size(), (size_t)(o.curve_off[r + 1] - o.curve_off[r]));
        for (size_t k = 0; k < g[r].curves.size(); k++) {
            const CurveSegment &s = g[r].curves[k];
            const float got[8] = {s.p0.first, s.p0.second, s.p1.first, s.p1.second,
                                  s.p2.first, s.p2.second, s.p3.first, s.p3.second};
            CHECK_EQ(std::memcmp(got, o.curve[o.curve_off[r] + k].p, 32), 0);
            CHECK_EQ(s.color.index, o.curve_color[o.curve_off[r] + k]);
        }
    }
}

void parity_case(int kind, uint64_t n, uint64_t seed) {
    std::vector<float> band;
    const std::vector<CommitInfo> commits = synth_list(kind, n, seed, &band);
    GraphLayout layout;
    layout.build(commits);
    CommitSoA soa(commits);
    wg_commits in = soa.view();
    wgo_layout L;
    CHECK_EQ(wgo_layout_build(&in, &L), 0);
    CHECK_EQ(layout.max_lane, (size_t)L.max_lane);
    CHECK_EQ(layout.graph_width, L.graph_width);
    for (size_t r = 0; r < commits.size(); r++) {
        const CommitLayout *l = layout.get(commits[r].id);
        CHECK(l && l->lane == L.lane[r] && l->color.index == L.color[r]);
    }
    CHECK_EQ(layout.edges.size(), (size_t)L.n_edges);
    for (size_t k = 0; k < layout.edges.size(); k++) {
        const GraphEdge &e = layout.edges[k];
        const wg_edge &o = L.edges[k];
        CHECK(e.child_row == o.child_row && e.child_lane == o.child_lane && e.parent_row == o.parent_row &&
              e.parent_lane == o.parent_lane && e.color.index == o.color);
    }
    const std::vector<float> h = compute_row_heights(commits);
    CHECK(std::memcmp(h.data(), L.heights, h.size() * 4) == 0);
    same_geometry(layout.row_geometry, L.geom);
    // a frame: row_geometry_with_bands, then graph_cell's vertices
    const std::vector<RowGeometry> g = layout.row_geometry_with_bands(commits, band);
    wgo_geometry og;
    CHECK_EQ(wgo_row_geometry(&L, soa.time.data(), band.data(), &og), 0);
    same_geometry(g, og);
    const auto pal = default_palette();
    const int64_t sel = (int64_t)(n / 3);
    const wg_vertex_summary vs = layout.emit_vertices(0, n, sel, pal);
    wg_vertex *ov = nullptr;
    uint64_t *ooff = nullptr, on = 0;
    CHECK_EQ(wgo_emit_vertices(&L, &og, 0, n, sel, pal.data(), &ov, &ooff, &on), 0);
    CHECK_EQ(vs.n_vertices, on);
    CHECK_EQ(vs.checksum, wgo_vertex_checksum(ov, on));
    const std::vector<wg_vertex> v = layout.vertices();
    CHECK(std::memcmp(v.data(), ov, on * sizeof(wg_vertex)) == 0);   // positions 0 ulp
    wgo_free(ov);
    wgo_free(ooff);
    wgo_geometry_free(&og);
    wgo_layout_free(&L);
}

}  // namespace

TEST(parity_linear_c1_shape) { parity_case(WGS_LINEAR, 10'000, 0x5EED + 1); }
TEST(parity_random13_c3_shape) { parity_case(WGS_RANDOM13, 20'000, 0x5EED + 3); }
TEST(parity_linux_c4_shape) { parity_case(WGS_LINUX, 20'000, 0x5EED + 4); }
TEST(parity_wide16_c5_shape) { parity_case(WGS_WIDE16, 20'000, 0x5EED + 5); }
TEST(parity_anomalies) { parity_case(WGS_ANOMALY, 5'000, 77); }

int main(int argc, char **argv) {
    std::vector<std::string> want;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--list") {
            for (auto &t : registry()) std::printf("%s\n", t.first.c_str());
            return 0;
        }
        if (a == "--no-device") {   // CPU box: the engine refuses, nothing falls back to the host
            try {
                GraphLayout layout;
                std::printf("FAIL: GraphLayout constructed without a GPU\n");
                return 1;
            } catch (const Error &e) {
                std::printf("refused: status %d: %s\n", e.status(), e.what());
                return e.status() == WG_E_NODEVICE ? 0 : 1;
            }
        }
        want.push_back(a);
    }
    int failed = 0, ran = 0;
    for (auto &t : registry()) {
        if (!want.empty() && std::find(want.begin(), want.end(), t.first) == want.end()) continue;
        ran++;
        try {
            t.second();
            std::printf("ok   %s\n", t.first.c_str());
        } catch (const Failure &f) {
            failed++;
            std::printf("FAIL %s: %s\n", t.first.c_str(), f.what.c_str());
        } catch (const std::exception &e) {
            failed++;
            std::printf("FAIL %s: exception: %s\n", t.first.c_str(), e.what());
        }
        std::fflush(stdout);
    }
    std::printf("%d of %d tests passed\n", ran - failed, ran);
    return failed ? 1 : 0;
}
