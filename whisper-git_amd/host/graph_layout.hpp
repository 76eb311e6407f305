// graph_layout.hpp — C++ host side of the engine, mirroring the reference's
// `GraphLayout` interface (/root/reference/src/commit_graph.rs:162-507).
//
// The reference is a Rust crate; its drop-in is a Rust shim over the C ABI
// (INTEGRATION.md §3).  No Rust toolchain exists in this image, so this is
// the same shim in C++: the same type names, fields, methods and argument
// meaning, implemented over include/wgraph.h (every computation runs in the
// HIP engine; nothing here restates the algorithm).  Parity tests written
// against it (tests/cpp/test_graph_layout.cpp) read like the reference's own
// tests (commit_graph.rs:1585-1763).
//
// Differences forced by the boundary, and only these:
//  - Colour is the palette index the engine carries (WG_COLOR_*), not an
//    aetna theme token; LANE_COLORS[i] = {i}, ORPHAN_COLOR = {6}.
//  - The reference is infallible.  The engine can fail (no gfx950 device,
//    out of device memory): every method then throws wgraph::Error carrying
//    the ABI status and wg_last_error().  There is no CPU fallback.
//  - row_geometry_with_bands(commits, bands) computes heights from `commits`
//    in the reference; the engine holds the built list's times on the
//    device, so `commits` must be that list (same length and times) —
//    anything else throws std::invalid_argument (the reference would index
//    its own edges into a different list).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "wgraph.h"

namespace wgraph {

// git2::Oid (20 bytes)
struct Oid {
    std::array<uint8_t, 20> bytes{};
    static Oid zero() { return Oid{}; }
    bool operator==(const Oid &o) const { return bytes == o.bytes; }
    bool operator!=(const Oid &o) const { return bytes != o.bytes; }
};

struct OidHash {
    size_t operator()(const Oid &o) const noexcept {
        uint64_t h = 1469598103934665603ull;   // FNV-1a
        for (uint8_t b : o.bytes) h = (h ^ b) * 1099511628211ull;
        return (size_t)h;
    }
};

// aetna Color token, carried as the engine's palette index (wgraph.h)
struct Color {
    uint8_t index = 0;
    bool operator==(const Color &o) const { return index == o.index; }
    bool operator!=(const Color &o) const { return index != o.index; }
};
inline constexpr Color LANE_COLORS[6] = {{0}, {1}, {2}, {3}, {4}, {5}};   // :59-66
inline constexpr Color ORPHAN_COLOR{WG_COLOR_ORPHAN};                     // :70
inline constexpr Color FOREGROUND{WG_COLOR_FOREGROUND};                   // tokens::FOREGROUND, :898

inline constexpr float ROW_HEIGHT = WG_ROW_HEIGHT;                // :30
inline constexpr float LANE_W = WG_LANE_W;                        // :33
inline constexpr size_t LANE_COUNT_VISUAL = WG_LANE_COUNT_VISUAL; // :37
inline constexpr float NODE_Y = WG_NODE_Y;                        // :43
inline constexpr float MAX_EXTRA_HEIGHT = WG_MAX_EXTRA_HEIGHT;    // :47
inline constexpr float PILLS_BAND_HEIGHT = WG_PILLS_BAND_HEIGHT;  // :106

// CommitInfo (git/mod.rs:246-270): the fields the layout path reads
struct CommitInfo {
    Oid id;
    std::string short_id;
    std::string summary;
    std::string author;
    int64_t time = 0;
    std::vector<Oid> parent_ids;
    bool is_synthetic = false;
    bool is_orphaned = false;
};

// :162-166
struct CommitLayout {
    size_t lane = 0;
    Color color;
};

// :173-180
struct GraphEdge {
    size_t child_row = 0;
    size_t child_lane = 0;
    size_t parent_row = 0;
    size_t parent_lane = 0;
    Color color;
};

// :186-193 (x in lane units, y row-local pixels)
struct CurveSegment {
    std::pair<float, float> p0, p1, p2, p3;
    Color color;
};

// :208-233 (Default: height ROW_HEIGHT, node_y NODE_Y)
struct RowGeometry {
    float height = ROW_HEIGHT;
    std::vector<std::pair<size_t, Color>> full_verticals;
    std::vector<std::pair<size_t, Color>> top_half_verticals;
    std::vector<std::pair<size_t, Color>> bottom_half_verticals;
    std::vector<CurveSegment> curves;
    float node_y = NODE_Y;
};

// An engine failure (status = WG_E_*; message from wg_last_error).
class Error : public std::runtime_error {
public:
    Error(int status, const std::string &msg) : std::runtime_error(msg), status_(status) {}
    int status() const { return status_; }

private:
    int status_;
};

// One engine context (wg_create / wg_destroy); one per calling thread.
class Engine {
public:
    explicit Engine(int device = 0);
    wg_ctx *get() const { return ctx_.get(); }
    void check(int rc, const char *what) const;   // throws Error when rc != WG_OK

private:
    std::unique_ptr<wg_ctx, void (*)(wg_ctx *)> ctx_;
};

// The commit list as the engine's structure-of-arrays (wg_commits, host).
struct CommitSoA {
    std::vector<uint8_t> oid, parent_oid, flags;
    std::vector<int64_t> time;
    std::vector<uint32_t> parent_off;
    explicit CommitSoA(const std::vector<CommitInfo> &commits);
    wg_commits view() const;
};

// GraphLayout (:240-472)
class GraphLayout {
public:
    GraphLayout();                    // GraphLayout::new (:261); device 0
    explicit GraphLayout(int device);

    // :265-355 — lanes, colours, edges and the default row geometry
    void build(const std::vector<CommitInfo> &commits);
    // :357 — the layout of the last row holding `id` (HashMap insert order)
    const CommitLayout *get(const Oid &id) const;
    // :367-399 — band_heights[i] (missing entries = 0) above row i.  Not
    // const, unlike the reference's `&self`: the engine's current geometry
    // becomes the banded one, so emit_vertices() draws it afterwards (the
    // pub field row_geometry keeps the build's copy).
    std::vector<RowGeometry> row_geometry_with_bands(const std::vector<CommitInfo> &commits,
                                                     const std::vector<float> &band_heights);

    // pub fields (:244-257)
    size_t max_lane = 0;
    std::vector<GraphEdge> edges;
    std::vector<RowGeometry> row_geometry;
    float graph_width = 0.0f;

    // Beyond the reference's surface: the engine behind it.  graph_cell's
    // tessellated output (WG-TESS-1) for rows [row_begin, row_end) of the
    // geometry of the last build / row_geometry_with_bands call.
    wg_vertex_summary emit_vertices(uint64_t row_begin, uint64_t row_end, int64_t selected_row,
                                    const std::array<float, 4 * WG_PALETTE_SIZE> &palette) const;
    std::vector<wg_vertex> vertices() const;   // the last emission, copied to the host
    wg_ctx *ctx() const { return eng_.get(); }

private:
    std::vector<RowGeometry> copy_geometry() const;

    Engine eng_;
    std::unordered_map<Oid, CommitLayout, OidHash> layouts_;
    std::vector<int64_t> time_;   // the built list's times
    mutable uint64_t n_vtx_ = 0;
};

// compute_row_heights (:486-507), on the calling thread's engine context
std::vector<float> compute_row_heights(const std::vector<CommitInfo> &commits);

// Default palette for emit_vertices: the dark theme's RGBA for the tokens
// LANE_COLORS / ORPHAN_COLOR / FOREGROUND name (wgraph.abi.DEFAULT_PALETTE);
// consumers pass their theme's.
std::array<float, 4 * WG_PALETTE_SIZE> default_palette();

}  // namespace wgraph
