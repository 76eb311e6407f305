// graph_layout.cpp — GraphLayout (commit_graph.rs:240-507) over the C ABI.
// Marshalling only: the list goes to the engine as structure-of-arrays, the
// engine's outputs come back into the reference's types.
#include "graph_layout.hpp"

#include <cstring>

namespace wgraph {

Engine::Engine(int device) : ctx_(wg_create(device), wg_destroy) {
    if (!ctx_) throw Error(WG_E_NODEVICE, "wg_create: no gfx950 device or the engine's code object did not load");
}

void Engine::check(int rc, const char *what) const {
    if (rc != WG_OK) throw Error(rc, std::string(what) + ": " + wg_last_error(ctx_.get()));
}

CommitSoA::CommitSoA(const std::vector<CommitInfo> &commits) {
    const size_t n = commits.size();
    oid.resize(n * 20);
    time.resize(n);
    flags.resize(n);
    parent_off.resize(n + 1);
    size_t e = 0;
    for (const CommitInfo &c : commits) e += c.parent_ids.size();
    parent_oid.resize(e * 20);
    size_t k = 0;
    for (size_t i = 0; i < n; i++) {
        const CommitInfo &c = commits[i];
        std::memcpy(&oid[i * 20], c.id.bytes.data(), 20);
        time[i] = c.time;
        flags[i] = (uint8_t)((c.is_orphaned ? WG_FLAG_ORPHAN : 0u) | (c.is_synthetic ? WG_FLAG_SYNTHETIC : 0u));
        parent_off[i] = (uint32_t)k;
        for (const Oid &p : c.parent_ids) std::memcpy(&parent_oid[20 * k++], p.bytes.data(), 20);
    }
    parent_off[n] = (uint32_t)k;
}

wg_commits CommitSoA::view() const {
    wg_commits c{};
    c.n_commits = time.size();
    c.n_parents = parent_off.back();
    c.oid = oid.data();
    c.time = time.data();
    c.parent_off = parent_off.data();
    c.parent_oid = parent_oid.data();
    c.flags = flags.data();
    c.residency = WG_HOST;
    return c;
}

GraphLayout::GraphLayout() : GraphLayout(0) {}
GraphLayout::GraphLayout(int device) : eng_(device) {}

void GraphLayout::build(const std::vector<CommitInfo> &commits) {
    if (commits.size() >= (1ull << 32) || [&] {
            size_t e = 0;
            for (const CommitInfo &c : commits) e += c.parent_ids.size();
            return e >= (1ull << 32);
        }())
        throw Error(WG_E_UNSUPPORTED, "build: more than 2^32 - 1 rows or parent references");
    layouts_.clear();
    edges.clear();
    row_geometry.clear();
    max_lane = 0;
    const CommitSoA soa(commits);
    const wg_commits in = soa.view();
    eng_.check(wg_layout_build(eng_.get(), &in), "wg_layout_build");
    time_ = soa.time;

    wg_layout_summary s{};
    eng_.check(wg_layout_summary_get(eng_.get(), &s), "wg_layout_summary_get");
    max_lane = s.max_lane;
    graph_width = s.graph_width;

    const size_t n = commits.size();
    std::vector<uint32_t> lane(n);
    std::vector<uint8_t> color(n);
    if (n) eng_.check(wg_copy_lanes(eng_.get(), lane.data(), color.data()), "wg_copy_lanes");
    // self.layouts.insert(commit.id, ...) in row order: the last row holding an id wins
    layouts_.reserve(n);
    for (size_t i = 0; i < n; i++) layouts_[commits[i].id] = CommitLayout{lane[i], Color{color[i]}};

    std::vector<wg_edge> e(s.n_edges);
    if (!e.empty()) eng_.check(wg_copy_edges(eng_.get(), e.data()), "wg_copy_edges");
    edges.reserve(e.size());
    for (const wg_edge &x : e)
        edges.push_back(GraphEdge{x.child_row, x.child_lane, x.parent_row, x.parent_lane, Color{(uint8_t)x.color}});

    row_geometry = copy_geometry();
}

const CommitLayout *GraphLayout::get(const Oid &id) const {
    const auto it = layouts_.find(id);
    return it == layouts_.end() ? nullptr : &it->second;
}

std::vector<RowGeometry> GraphLayout::row_geometry_with_bands(const std::vector<CommitInfo> &commits,
                                                              const std::vector<float> &band_heights) {
    // heights from the passed list (compute_row_heights(commits), :372), edges from
    // the built layout: wg_row_geometry_list; a list of another length is refused
    // by the engine (WG_E_INVALID, thrown as Error), never replaced by the built list
    std::vector<int64_t> t(commits.size());
    for (size_t i = 0; i < commits.size(); i++) t[i] = commits[i].time;
    wg_commits in{};
    in.n_commits = commits.size();
    in.time = t.data();
    in.residency = WG_HOST;
    // band_heights.get(i).copied().unwrap_or(0.0) (:375, :386)
    std::vector<float> band(commits.size(), 0.0f);
    std::memcpy(band.data(), band_heights.data(), std::min(band.size(), band_heights.size()) * sizeof(float));
    eng_.check(wg_row_geometry_list(eng_.get(), &in, band.data(), WG_HOST), "wg_row_geometry_list");
    return copy_geometry();
}

std::vector<RowGeometry> GraphLayout::copy_geometry() const {
    wg_geometry_summary gs{};
    eng_.check(wg_geometry_summary_get(eng_.get(), &gs), "wg_geometry_summary_get");
    const size_t n = gs.n_rows;
    std::vector<float> height(n), node_y(n), row_top(n + 1);
    std::vector<uint32_t> vert_off(n + 1), vert(gs.n_vert + 1), curve_off(n + 1);
    std::vector<wg_curve> curve(gs.n_curve + 1);
    std::vector<uint8_t> curve_color(gs.n_curve + 1);
    wg_geometry_host dst{height.data(), node_y.data(), row_top.data(), vert_off.data(),
                         vert.data(),   curve_off.data(), curve.data(), curve_color.data()};
    eng_.check(wg_copy_geometry(eng_.get(), &dst), "wg_copy_geometry");
    std::vector<RowGeometry> rows(n);
    for (size_t r = 0; r < n; r++) {
        RowGeometry &g = rows[r];
        g.height = height[r];
        g.node_y = node_y[r];
        for (uint32_t k = vert_off[r]; k < vert_off[r + 1]; k++) {
            const uint32_t v = vert[k];
            const std::pair<size_t, Color> entry{WG_VERT_LANE(v), Color{(uint8_t)WG_VERT_COLOR(v)}};
            switch (WG_VERT_KIND(v)) {
            case WG_VERT_FULL: g.full_verticals.push_back(entry); break;
            case WG_VERT_TOP: g.top_half_verticals.push_back(entry); break;
            default: g.bottom_half_verticals.push_back(entry); break;
            }
        }
        for (uint32_t k = curve_off[r]; k < curve_off[r + 1]; k++) {
            const float *p = curve[k].p;
            g.curves.push_back(CurveSegment{{p[0], p[1]}, {p[2], p[3]}, {p[4], p[5]}, {p[6], p[7]}, Color{curve_color[k]}});
        }
    }
    return rows;
}

wg_vertex_summary GraphLayout::emit_vertices(uint64_t row_begin, uint64_t row_end, int64_t selected_row,
                                             const std::array<float, 4 * WG_PALETTE_SIZE> &palette) const {
    eng_.check(wg_emit_vertices(eng_.get(), row_begin, row_end, selected_row, palette.data()), "wg_emit_vertices");
    wg_vertex_summary s{};
    eng_.check(wg_vertex_summary_get(eng_.get(), &s), "wg_vertex_summary_get");
    n_vtx_ = s.n_vertices;
    return s;
}

std::vector<wg_vertex> GraphLayout::vertices() const {
    std::vector<wg_vertex> v(n_vtx_);
    if (n_vtx_) eng_.check(wg_copy_vertices(eng_.get(), 0, n_vtx_, v.data()), "wg_copy_vertices");
    return v;
}

std::vector<float> compute_row_heights(const std::vector<CommitInfo> &commits) {
    thread_local std::unique_ptr<Engine> eng;   // one context per calling thread (wgraph.h)
    if (!eng) eng = std::make_unique<Engine>(0);
    std::vector<int64_t> t(commits.size());
    for (size_t i = 0; i < commits.size(); i++) t[i] = commits[i].time;
    std::vector<float> h(commits.size());
    eng->check(wg_compute_row_heights(eng->get(), t.data(), t.size(), WG_HOST, h.data()), "wg_compute_row_heights");
    return h;
}

std::array<float, 4 * WG_PALETTE_SIZE> default_palette() {
    return {0.231f, 0.510f, 0.965f, 1.0f,    // PRIMARY
            0.133f, 0.773f, 0.369f, 1.0f,    // SUCCESS
            0.961f, 0.620f, 0.043f, 1.0f,    // WARNING
            0.024f, 0.714f, 0.831f, 1.0f,    // INFO
            0.937f, 0.267f, 0.267f, 1.0f,    // DESTRUCTIVE
            0.898f, 0.906f, 0.922f, 1.0f,    // FOREGROUND (lane 5)
            0.612f, 0.639f, 0.686f, 1.0f,    // MUTED_FOREGROUND (orphan)
            0.898f, 0.906f, 0.922f, 1.0f};   // FOREGROUND (selected ring)
}

}  // namespace wgraph
