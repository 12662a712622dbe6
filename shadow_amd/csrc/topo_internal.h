// topo_internal.h -- host-side data structures shared by the libshdtopo translation units.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "topo_device.h"

namespace shdtopo {

// Page-locked host memory for the arrays the graph preparation uploads (topo_core.cpp
// upload_csr): the copy is then a DMA at PCIe speed instead of the runtime's staged pageable
// copy.  Ordinary memory when no GPU is present (the CPU-only parser and tests).
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) {}
    T* allocate(size_t n) {
        void* p = pinned_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { pinned_free(p); }
    template <class U>
    bool operator==(const PinnedAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
template <class T>
using PinnedVec = std::vector<T, PinnedAlloc<T>>;

// The parsed topology: what igraph_read_graph_graphml + the C attribute table hold for the
// reference (shd-topology.c:95-123).  Vertex index = order of first appearance of the node id,
// edge id = order of <edge> elements (igraph 0.7.1 GraphML reader).
struct HostGraph {
    int32_t V = 0;
    int64_t E = 0;
    bool directed = false;
    PinnedVec<int32_t> eu, ev;             // endpoints in document order
    PinnedVec<double> elat, eloss;
    std::vector<double> ejitter;
    std::vector<std::string> vid, vtype, vip, vgeo;
    std::vector<double> vbwup, vbwdown, vloss;
};

bool graphml_parse(const char* buf, size_t len, HostGraph& g, std::string& err);
bool graphml_load_file(const char* path, HostGraph& g, std::string& err);
bool graphml_write_file(const HostGraph& g, const char* path);

struct SynthParams {
    uint64_t seed;
    int64_t n_routers, n_poi, n_edges;
    int integer_latency;
    double alpha;
    int directed = 0;
};
bool synth_graph(const SynthParams& p, HostGraph& g, std::string& err);

// splitmix64: the generators' deterministic RNG
struct SplitMix {
    uint64_t s;
    explicit SplitMix(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    uint64_t below(uint64_t n) { return next() % n; }
};

// glibc rand_r (the generator behind src/utility/shd-random.c:30-37)
inline int32_t glibc_rand_r(uint32_t* seed) {
    uint32_t next = *seed;
    int32_t result;
    next = next * 1103515245u + 12345u;
    result = (int32_t)((next / 65536u) % 2048u);
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    *seed = next;
    return result;
}
inline double rand_r_double(uint32_t* seed) { return (double)glibc_rand_r(seed) / 2147483647.0; }

// Host side of the graph preparation (topo_core.cpp upload_csr), relabelled ids.
struct HostPrep {
    std::vector<int32_t> perm;      // new -> old
    std::vector<int32_t> inv;       // old -> new
    std::vector<double> pot;        // pi = d(h0, v) from the top hub: bucket shifts, batch order
    std::vector<uint32_t> sptPar;   // h0 shortest-path tree parent (source ordering)
    // preorder of the parent forest (roots and children by ascending id, so h0 = vertex 0's tree
    // comes first) and each vertex's depth below its root (tree_order): the source grouping and
    // the batch order of a cold build read them instead of walking every source's parent path
    std::vector<uint32_t> preorder, depth;
    double piMax = 0.0;             // largest finite pi
    // directed topologies: d(v, h0) over the in-rows (undirected: empty, pot serves), the bucket
    // shifts' value of d_s(h0), and its largest finite value
    std::vector<double> potSrc;
    double srcMax = 0.0;
    double to_h0(uint32_t v) const { return potSrc.empty() ? pot[v] : potSrc[v]; }
    double to_h0_max() const { return potSrc.empty() ? piMax : srcMax; }
};

// HostPrep::preorder / depth from sptPar (O(V); runs with the graph preparation)
inline void tree_order(HostPrep& hp) {
    const uint32_t V = (uint32_t)hp.sptPar.size();
    std::vector<uint32_t> cstart((size_t)V + 1, 0), child, fill;
    for (uint32_t v = 0; v < V; v++) {
        const uint32_t p = hp.sptPar[v];
        if (p < V) cstart[(size_t)p + 1]++;
    }
    for (uint32_t v = 0; v < V; v++) cstart[(size_t)v + 1] += cstart[v];
    child.resize(cstart[V]);
    fill.assign(cstart.begin(), cstart.end() - 1);
    for (uint32_t v = 0; v < V; v++) {  // children in ascending id order
        const uint32_t p = hp.sptPar[v];
        if (p < V) child[fill[p]++] = v;
    }
    hp.preorder.assign(V, 0xFFFFFFFFu);
    hp.depth.assign(V, 0);
    std::vector<uint32_t> stack;
    uint32_t next = 0;
    for (uint32_t r = 0; r < V; r++) {
        if (hp.sptPar[r] < V) continue;  // roots in ascending id order: h0's tree first
        stack.push_back(r);
        while (!stack.empty()) {
            const uint32_t v = stack.back();
            stack.pop_back();
            hp.preorder[v] = next++;
            for (uint32_t k = cstart[(size_t)v + 1]; k > cstart[v]; k--) {  // smallest id on top
                const uint32_t c = child[k - 1];
                hp.depth[c] = hp.depth[v] + 1;
                stack.push_back(c);
            }
        }
    }
    // a vertex on a parent cycle (no root above it) keeps the walk's cap, V + 1 hops, and sorts
    // last in its input order (preorder stays UINT32_MAX)
    for (uint32_t v = 0; v < V; v++)
        if (hp.preorder[v] == 0xFFFFFFFFu) hp.depth[v] = V + 1;
}

uint32_t string_to_ip(const char* s);  // inet_pton(AF_INET) as shd-address.c:137-144

// Host view of one device routing table for the per-call getters: the column map it was built
// for and the row minima (immutable), plus the rows the getters have read so far.  A row's
// {latency, reliability} records are copied from the device table the first time a query needs
// them (16 A bytes, C4: 160 KB) and published with a release store; readers never lock.  A full
// A x A mirror is never made (round 5 copied all 1.8 GB at C4 before the first answer).
struct HostTable {
    uint64_t gen = 0;     // attached-set generation (Topology::setGen) of the table
    uint64_t serial = 0;  // Topology::tableSerial of the table (every build / bind bumps it)
    uint64_t epoch = 0;   // attach epoch (Topology::ipGen) of its columns: a row materialised
                          // from this table covers the vertices attached at that epoch
    int64_t A = 0;
    std::shared_ptr<const std::vector<int32_t>> colOf;  // shared by snapshots of one geometry
    std::vector<double> rowmin;
    // per column: its row, nullptr until first read (published once, compare-exchange)
    std::unique_ptr<std::atomic<const double2*>[]> rows;
    mutable std::vector<std::unique_ptr<double2[]>> rowStore;  // owner of the copied rows
    mutable std::mutex storeMu;                                // (guards rowStore)
    int32_t col(int32_t v) const { return (*colOf)[(size_t)v]; }
};

// Index of the attachment candidates (the "poi" vertices) so that attaching H hosts costs
// O(H + V) instead of the reference's O(H * V) string scan (shd-topology.c:1087); candidate
// lists keep vertex order, so the chosen vertex and RNG use are identical.
struct AttachIndex {
    bool built = false;
    std::vector<int32_t> all;                                   // poi vertices, index order
    std::vector<uint32_t> ip;                                   // per vertex (poi only)
    std::vector<uint8_t> usable;                                // per vertex
    std::unordered_map<std::string, std::vector<int32_t>> byType, byCode, byTypeCode;
    std::unordered_map<uint32_t, std::vector<int32_t>> byIP;
    void build(const HostGraph& g);
};

}  // namespace shdtopo
