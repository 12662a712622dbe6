// topo_graph.cpp -- GraphML reader/writer and the synthetic topology generator.
//
// The reader restates what Shadow gets from igraph 0.7.1's igraph_read_graph_graphml
// (called at src/topology/shd-topology.c:110): vertex index = order of first appearance of
// the node id, edge id = <edge> order, numeric keys (int/long/float/double) -> f64 via a
// correctly rounded decimal parse (strtod), a missing numeric value -> NaN (or the key's
// <default>), a missing string -> "" (or <default>).  It is a dedicated single-pass tokenizer
// (no DOM) so the 1M-vertex synthetic files ("hard parts") load in seconds.
#include <arpa/inet.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <charconv>
#include <functional>
#include <memory>
#include <thread>

#include "topo_internal.h"

namespace shdtopo {

uint32_t string_to_ip(const char* s) {
    if (!s) return 0xFFFFFFFFu;  // INADDR_NONE
    struct in_addr a;
    if (inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return 0xFFFFFFFFu;
}

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

struct Span {
    const char* b = nullptr;
    const char* e = nullptr;
    size_t size() const { return (size_t)(e - b); }
    bool eq(const char* s) const {
        const size_t n = strlen(s);
        return size() == n && !memcmp(b, s, n);
    }
    bool eq(const std::string& s) const { return size() == s.size() && !memcmp(b, s.data(), s.size()); }
    std::string str() const { return std::string(b, e); }
};

void decode_entities_into(const char* b, const char* e, std::string& out) {
    out.clear();
    out.reserve((size_t)(e - b));
    for (const char* p = b; p < e; ++p) {
        if (*p != '&') { out.push_back(*p); continue; }
        const char* q = (const char*)memchr(p, ';', (size_t)(e - p));
        if (!q) { out.push_back(*p); continue; }
        std::string ent(p + 1, q);
        if (ent == "lt") out.push_back('<');
        else if (ent == "gt") out.push_back('>');
        else if (ent == "amp") out.push_back('&');
        else if (ent == "quot") out.push_back('"');
        else if (ent == "apos") out.push_back('\'');
        else if (!ent.empty() && ent[0] == '#') {
            unsigned long cp = (ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X'))
                                   ? strtoul(ent.c_str() + 2, nullptr, 16)
                                   : strtoul(ent.c_str() + 1, nullptr, 10);
            if (cp < 0x80) out.push_back((char)cp);
            else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
            else if (cp < 0x10000) { out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F))); }
            else { out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 0x3F))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F))); }
        } else { out.append(p, q + 1); }
        p = q;
    }
}

// A tag as spans into the buffer: no allocation per tag.  Attribute values that contain an
// entity are decoded on demand (value()).
struct Tag {
    Span name;  // local name (namespace prefix stripped)
    bool closing = false, selfclose = false;
    int nattr = 0;
    Span an[16], av[16];
    const Span* attr(const char* k) const {
        for (int i = 0; i < nattr; i++)
            if (an[i].eq(k)) return &av[i];
        return nullptr;
    }
};

inline std::string value(const Span& s) {
    std::string out;
    if (memchr(s.b, '&', s.size())) decode_entities_into(s.b, s.e, out);
    else out.assign(s.b, s.e);
    return out;
}

// parse one tag starting at p ('<'), return pointer past '>' or nullptr
const char* parse_tag(const char* p, const char* end, Tag& t) {
    t.nattr = 0;
    t.closing = t.selfclose = false;
    ++p;
    if (p < end && *p == '/') { t.closing = true; ++p; }
    const char* nb = p;
    while (p < end && !is_space(*p) && *p != '>' && *p != '/') ++p;
    const char* colon = (const char*)memchr(nb, ':', (size_t)(p - nb));
    t.name.b = colon ? colon + 1 : nb;
    t.name.e = p;
    for (;;) {
        while (p < end && is_space(*p)) ++p;
        if (p >= end) return nullptr;
        if (*p == '>') return p + 1;
        if (*p == '/') {
            t.selfclose = true;
            while (p < end && *p != '>') ++p;
            return p < end ? p + 1 : nullptr;
        }
        const char* kb = p;
        while (p < end && *p != '=' && !is_space(*p) && *p != '>') ++p;
        Span k{kb, p}, v{p, p};
        while (p < end && is_space(*p)) ++p;
        if (p < end && *p == '=') {
            ++p;
            while (p < end && is_space(*p)) ++p;
            if (p >= end) return nullptr;
            const char q = *p;
            if (q != '"' && q != '\'') return nullptr;
            ++p;
            const char* ve = (const char*)memchr(p, q, (size_t)(end - p));
            if (!ve) return nullptr;
            v = Span{p, ve};
            p = ve + 1;
        }
        if (t.nattr < 16) {
            t.an[t.nattr] = k;
            t.av[t.nattr] = v;
            t.nattr++;
        }
    }
}

// strtod on a span (correctly rounded in glibc), leading blanks skipped; no digits -> NaN
double parse_numeric(const char* b, const char* e) {
    while (b < e && is_space(*b)) ++b;
    if (b >= e) return NAN;
    char tmp[64];
    const size_t n = (size_t)(e - b);
    std::string big;
    const char* c;
    if (n < sizeof tmp) {
        memcpy(tmp, b, n);
        tmp[n] = 0;
        c = tmp;
    } else {
        big.assign(b, e);
        c = big.c_str();
    }
    char* endp = nullptr;
    const double v = strtod(c, &endp);
    return endp == c ? NAN : v;
}
double parse_numeric(const std::string& s) { return parse_numeric(s.data(), s.data() + s.size()); }

// open-addressing map node id (span into the buffer, or an owned decoded copy) -> vertex
struct IdMap {
    std::vector<int32_t> slot;  // -1 = empty
    std::vector<Span> keys;     // per vertex
    std::vector<std::unique_ptr<std::string>> owned;
    size_t mask = 0;
    static uint64_t hash(const Span& s) {
        uint64_t h = 1469598103934665603ull;
        for (const char* c = s.b; c < s.e; ++c) h = (h ^ (uint8_t)*c) * 1099511628211ull;
        return h ^ (h >> 29);
    }
    void grow() {
        const size_t cap = slot.empty() ? (1u << 16) : slot.size() * 2;
        slot.assign(cap, -1);
        mask = cap - 1;
        for (size_t v = 0; v < keys.size(); v++) {
            size_t i = hash(keys[v]) & mask;
            while (slot[i] >= 0) i = (i + 1) & mask;
            slot[i] = (int32_t)v;
        }
    }
    int32_t find(const Span& s) const {
        if (slot.empty()) return -1;
        size_t i = hash(s) & mask;
        while (slot[i] >= 0) {
            const Span& k = keys[(size_t)slot[i]];
            if (k.size() == s.size() && !memcmp(k.b, s.b, s.size())) return slot[i];
            i = (i + 1) & mask;
        }
        return -1;
    }
    // returns (vertex, created)
    std::pair<int32_t, bool> find_or_add(Span s, bool needs_decode) {
        if (needs_decode) {
            owned.emplace_back(new std::string());
            decode_entities_into(s.b, s.e, *owned.back());
            s = Span{owned.back()->data(), owned.back()->data() + owned.back()->size()};
        }
        if ((keys.size() + 1) * 2 > slot.size()) grow();
        size_t i = hash(s) & mask;
        while (slot[i] >= 0) {
            const Span& k = keys[(size_t)slot[i]];
            if (k.size() == s.size() && !memcmp(k.b, s.b, s.size())) {
                if (needs_decode) owned.pop_back();
                return {slot[i], false};
            }
            i = (i + 1) & mask;
        }
        slot[i] = (int32_t)keys.size();
        keys.push_back(s);
        return {(int32_t)keys.size() - 1, true};
    }
};

struct Key {
    std::string id, name, type, forwhat, def;
    bool has_default = false;
};

// attributes of the reference's schema (shd-topology.c:220-372): vertex type/ip/geocode (string),
// bandwidthup/bandwidthdown/packetloss (numeric); edge latency/jitter/packetloss (numeric)
enum VAttr { VA_TYPE, VA_IP, VA_GEO, VA_BWUP, VA_BWDOWN, VA_LOSS, VA_N };
enum EAttr { EA_LAT, EA_JIT, EA_LOSS, EA_N };

struct Schema {
    std::vector<Key> keys;
    std::vector<int> kslot_v, kslot_e;  // per key (document order): attribute it feeds or -1
    std::string vdef_s[3];
    double vdef_n[3] = {NAN, NAN, NAN}, edef[EA_N] = {NAN, NAN, NAN};
    bool resolved = false;
    // the first key (document order) of a name in the element's domain wins; its <default> is
    // what an element without that data element gets
    void resolve() {
        resolved = true;
        kslot_v.assign(keys.size(), -1);
        kslot_e.assign(keys.size(), -1);
        static const char* vn[VA_N] = {"type", "ip", "geocode", "bandwidthup", "bandwidthdown",
                                       "packetloss"};
        static const char* en[EA_N] = {"latency", "jitter", "packetloss"};
        for (int a = 0; a < VA_N; a++)
            for (size_t k = 0; k < keys.size(); k++) {
                const Key& K = keys[k];
                if ((K.forwhat == "all" || K.forwhat == "node") && K.name == vn[a]) {
                    if (kslot_v[k] < 0) kslot_v[k] = a;
                    if (a < 3) vdef_s[a] = K.has_default ? K.def : std::string();
                    else vdef_n[a - 3] = K.has_default ? parse_numeric(K.def) : NAN;
                    break;
                }
            }
        for (int a = 0; a < EA_N; a++)
            for (size_t k = 0; k < keys.size(); k++) {
                const Key& K = keys[k];
                if ((K.forwhat == "all" || K.forwhat == "edge") && K.name == en[a]) {
                    if (kslot_e[k] < 0) kslot_e[k] = a;
                    edef[a] = K.has_default ? parse_numeric(K.def) : NAN;
                    break;
                }
            }
    }
    int key_index(const Span& id) const {
        for (size_t k = 0; k < keys.size(); k++)
            if (id.eq(keys[k].id)) return (int)k;
        return -1;
    }
};

struct EdgeOut {
    std::vector<int32_t> eu, ev;
    std::vector<double> lat, jit, loss;
};

// One pass of the tokenizer over [p, end).  Full mode builds keys, vertices and edges in
// document order.  Edge-chunk mode (parallel edge section) only appends edges to its own
// EdgeOut, looking node ids up read-only: any construct it cannot handle there (a <node>, an id
// not seen before, a <key>, CDATA or a comment) makes it fail, and the caller re-parses
// sequentially.
struct Parser {
    Schema* sc;
    IdMap* ids;
    HostGraph* g;      // full mode: vertices (and edges via eo)
    EdgeOut* eo;
    bool chunk;        // edge-chunk mode
    std::string* err;
    bool failed = false;
    bool graph_seen = false;
    bool in_key = false, in_default = false;
    Key cur_key;
    std::string text, sval;
    enum { NONE, IN_NODE, IN_EDGE } ctx = NONE;
    int32_t cur_vertex = -1;

    bool fail(const char* m) {
        failed = true;
        if (!chunk && err) *err = m;
        return false;
    }
    int32_t vertex(const Span& id) {
        const bool dec = memchr(id.b, '&', id.size()) != nullptr;
        if (chunk) {
            const int32_t v = dec ? -1 : ids->find(id);
            if (v < 0) fail("edge chunk: unknown node id");
            return v;
        }
        const auto r = ids->find_or_add(id, dec);
        if (r.second) {
            g->V++;
            g->vtype.push_back(sc->vdef_s[VA_TYPE]);
            g->vip.push_back(sc->vdef_s[VA_IP]);
            g->vgeo.push_back(sc->vdef_s[VA_GEO]);
            g->vbwup.push_back(sc->vdef_n[VA_BWUP - 3]);
            g->vbwdown.push_back(sc->vdef_n[VA_BWDOWN - 3]);
            g->vloss.push_back(sc->vdef_n[VA_LOSS - 3]);
        }
        return r.second ? -(r.first + 2) : r.first;  // <= -2: created now
    }
    double num(const char* b, const char* e, bool decode) {
        if (!decode) return parse_numeric(b, e);
        decode_entities_into(b, e, sval);
        return parse_numeric(sval);
    }
    void store(int k, const char* b, const char* e, bool decode) {
        if (k < 0) return;
        if (ctx == IN_NODE && cur_vertex >= 0 && sc->kslot_v[(size_t)k] >= 0) {
            const int a = sc->kslot_v[(size_t)k];
            const size_t v = (size_t)cur_vertex;
            if (a < 3) {
                if (decode) decode_entities_into(b, e, sval); else sval.assign(b, e);
                (a == VA_TYPE ? g->vtype : a == VA_IP ? g->vip : g->vgeo)[v] = sval;
            } else {
                (a == VA_BWUP ? g->vbwup : a == VA_BWDOWN ? g->vbwdown : g->vloss)[v] = num(b, e, decode);
            }
        } else if (ctx == IN_EDGE && sc->kslot_e[(size_t)k] >= 0) {
            const int a = sc->kslot_e[(size_t)k];
            (a == EA_LAT ? eo->lat : a == EA_JIT ? eo->jit : eo->loss).back() = num(b, e, decode);
        }
    }
    // returns the position reached; *edge_at receives the start of the first <edge> tag when
    // stop_at_edge is set (full mode hands the edge section to the parallel chunks there)
    const char* run(const char* p, const char* end, bool stop_at_edge, const char** edge_at) {
        Tag t;
        while (p < end) {
            if (*p != '<') {
                const char* q = (const char*)memchr(p, '<', (size_t)(end - p));
                if (!q) q = end;
                if (in_default) text.append(p, q);
                p = q;
                continue;
            }
            if (end - p >= 4 && !memcmp(p, "<!--", 4)) {
                if (chunk) { fail("chunk: comment"); return p; }
                const char* q = strstr(p + 4, "-->");
                if (!q) { fail("unterminated comment"); return p; }
                p = q + 3;
                continue;
            }
            if (end - p >= 9 && !memcmp(p, "<![CDATA[", 9)) {
                if (chunk) { fail("chunk: CDATA"); return p; }
                const char* q = strstr(p + 9, "]]>");
                if (!q) { fail("unterminated CDATA"); return p; }
                if (in_default)  // CDATA text is literal: escape '&' for the entity decoder
                    for (const char* c = p + 9; c < q; ++c) {
                        if (*c == '&') text += "&amp;"; else text.push_back(*c);
                    }
                p = q + 3;
                continue;
            }
            if (end - p >= 2 && (p[1] == '?' || p[1] == '!')) {
                const char* q = (const char*)memchr(p, '>', (size_t)(end - p));
                if (!q) { fail("unterminated declaration"); return p; }
                p = q + 1;
                continue;
            }
            const char* tag0 = p;
            const char* nx = parse_tag(p, end, t);
            if (!nx) { fail("malformed tag"); return p; }
            const Span& nm = t.name;
            if (!t.closing && stop_at_edge && nm.eq("edge") && ctx == NONE) {
                *edge_at = tag0;
                return tag0;
            }
            p = nx;
            if (!t.closing) {
                if (nm.eq("data")) {
                    if (ctx != IN_NODE && ctx != IN_EDGE) continue;
                    const Span* ks = t.attr("key");
                    const int k = ks ? sc->key_index(*ks) : -1;
                    if (t.selfclose) { store(k, p, p, false); continue; }
                    // fast path: plain text up to </data>; otherwise collect CDATA / comments
                    const char* q = (const char*)memchr(p, '<', (size_t)(end - p));
                    if (!q) { fail("unterminated data"); return p; }
                    if (end - q >= 7 && !memcmp(q, "</data", 6) && (q[6] == '>' || is_space(q[6]))) {
                        store(k, p, q, memchr(p, '&', (size_t)(q - p)) != nullptr);
                        const char* gt = (const char*)memchr(q, '>', (size_t)(end - q));
                        if (!gt) { fail("malformed tag"); return p; }
                        p = gt + 1;
                        continue;
                    }
                    if (chunk) { fail("chunk: complex data"); return p; }
                    std::string acc;
                    for (;;) {
                        const char* r = (const char*)memchr(p, '<', (size_t)(end - p));
                        if (!r) { fail("unterminated data"); return p; }
                        acc.append(p, r);
                        p = r;
                        if (end - p >= 9 && !memcmp(p, "<![CDATA[", 9)) {
                            const char* c2 = strstr(p + 9, "]]>");
                            if (!c2) { fail("unterminated CDATA"); return p; }
                            for (const char* c = p + 9; c < c2; ++c) {
                                if (*c == '&') acc += "&amp;"; else acc.push_back(*c);
                            }
                            p = c2 + 3;
                        } else if (end - p >= 4 && !memcmp(p, "<!--", 4)) {
                            const char* c2 = strstr(p + 4, "-->");
                            if (!c2) { fail("unterminated comment"); return p; }
                            p = c2 + 3;
                        } else {
                            const char* gt = (const char*)memchr(p, '>', (size_t)(end - p));
                            if (!gt) { fail("malformed tag"); return p; }
                            p = gt + 1;  // </data> (or a stray tag inside data: ignored)
                            break;
                        }
                    }
                    store(k, acc.data(), acc.data() + acc.size(), true);
                } else if (nm.eq("edge")) {
                    const Span* sa = t.attr("source");
                    const Span* da = t.attr("target");
                    if (!sa || !da) { fail("edge without source/target"); return p; }
                    if (!sc->resolved) sc->resolve();
                    int32_t u = vertex(*sa);
                    if (failed) return p;
                    int32_t v = vertex(*da);
                    if (failed) return p;
                    eo->eu.push_back(u < -1 ? -(u + 2) : u);
                    eo->ev.push_back(v < -1 ? -(v + 2) : v);
                    eo->lat.push_back(sc->edef[EA_LAT]);
                    eo->jit.push_back(sc->edef[EA_JIT]);
                    eo->loss.push_back(sc->edef[EA_LOSS]);
                    if (!t.selfclose) ctx = IN_EDGE;
                } else if (chunk) {
                    if (!nm.eq("graph") && !nm.eq("graphml")) { fail("chunk: unexpected tag"); return p; }
                } else if (nm.eq("node")) {
                    const Span* id = t.attr("id");
                    if (!id) { fail("node without id"); return p; }
                    if (!sc->resolved) sc->resolve();
                    // first appearance creates the vertex; the data of an id seen before
                    // (declared again, or created by an earlier edge) is ignored, as the
                    // oracle's reader does
                    const int32_t r = vertex(*id);
                    cur_vertex = r < -1 ? -(r + 2) : -1;
                    if (!t.selfclose) ctx = IN_NODE;
                } else if (nm.eq("key")) {
                    cur_key = Key();
                    const Span* id = t.attr("id");
                    cur_key.id = id ? value(*id) : "";
                    const Span* an = t.attr("attr.name");
                    cur_key.name = an ? value(*an) : cur_key.id;
                    const Span* at = t.attr("attr.type");
                    cur_key.type = at ? value(*at) : "string";
                    const Span* fo = t.attr("for");
                    cur_key.forwhat = fo ? value(*fo) : "all";
                    if (t.selfclose) sc->keys.push_back(cur_key);
                    else in_key = true;
                } else if (nm.eq("default") && in_key) {
                    in_default = !t.selfclose;
                    text.clear();
                    if (t.selfclose) { cur_key.has_default = true; cur_key.def.clear(); }
                } else if (nm.eq("graph")) {
                    const Span* ed = t.attr("edgedefault");
                    // GraphML: edgedefault is required; igraph treats a missing one as directed
                    g->directed = !(ed && ed->eq("undirected"));
                    graph_seen = true;
                    sc->resolve();
                }
            } else {
                if (nm.eq("edge") && ctx == IN_EDGE) {
                    ctx = NONE;
                } else if (nm.eq("node") && ctx == IN_NODE) {
                    ctx = NONE;
                    cur_vertex = -1;
                } else if (nm.eq("key") && in_key) {
                    sc->keys.push_back(cur_key);
                    in_key = false;
                } else if (nm.eq("default") && in_default) {
                    decode_entities_into(text.data(), text.data() + text.size(), cur_key.def);
                    cur_key.has_default = true;
                    in_default = false;
                }
            }
        }
        return p;
    }
};

// the start of the first "<edge" tag at or after p (a tag name boundary), or end
const char* next_edge_tag(const char* p, const char* end) {
    while (p < end) {
        const char* q = (const char*)memchr(p, '<', (size_t)(end - p));
        if (!q) return end;
        if (end - q >= 6 && !memcmp(q + 1, "edge", 4) && (is_space(q[5]) || q[5] == '>' || q[5] == '/'))
            return q;
        p = q + 1;
    }
    return end;
}

}  // namespace

bool graphml_parse(const char* buf, size_t len, HostGraph& g, std::string& err) {
    g = HostGraph();
    Schema sc;
    IdMap ids;
    EdgeOut eo;
    const char* end = buf + len;
    Parser P{&sc, &ids, &g, &eo, false, &err};
    // 1) sequential: keys, the graph element, nodes -- up to the first <edge>
    const char* edge_at = nullptr;
    const char* p = P.run(buf, end, true, &edge_at);
    if (P.failed) return false;
    bool done = edge_at == nullptr;
    bool chunked = false;
    // 2) the edge section in parallel chunks split at <edge> tags (node ids are read-only now;
    //    anything unusual in a chunk makes the whole section fall back to the sequential pass)
    if (!done) {
        unsigned nt = std::thread::hardware_concurrency();
        if (const char* e = getenv("OMP_NUM_THREADS")) nt = std::min<unsigned>(nt, (unsigned)std::max(1, atoi(e)));
        nt = std::max(1u, std::min(nt, 32u));
        const size_t rem = (size_t)(end - p);
        if (!sc.resolved) sc.resolve();
        if (nt > 1 && rem > ((size_t)8 << 20)) {
            std::vector<const char*> cut{p};
            for (unsigned i = 1; i < nt; i++) {
                const char* c = next_edge_tag(std::max(cut.back() + 1, p + rem * i / nt), end);
                if (c >= end) break;
                cut.push_back(c);
            }
            cut.push_back(end);
            const size_t nc = cut.size() - 1;
            std::vector<EdgeOut> outs(nc);
            std::vector<char> bad(nc, 0);
            std::vector<std::thread> th;
            for (size_t c = 0; c < nc; c++)
                th.emplace_back([&, c]() {
                    Parser Q{&sc, &ids, nullptr, &outs[c], true, nullptr};
                    Q.graph_seen = true;
                    // a comment / CDATA section anywhere in the chunk (a cut may even fall inside
                    // one): leave the section to the sequential pass
                    if (memmem(cut[c], (size_t)(cut[c + 1] - cut[c]), "<!", 2)) {
                        bad[c] = 1;
                        return;
                    }
                    Q.run(cut[c], cut[c + 1], false, nullptr);
                    bad[c] = Q.failed || Q.ctx != Parser::NONE;  // a chunk must end between edges
                });
            for (auto& x : th) x.join();
            bool ok = true;
            for (size_t c = 0; c < nc; c++) ok = ok && !bad[c];
            if (ok) {
                size_t ne = eo.eu.size();
                for (auto& o : outs) ne += o.eu.size();
                // straight into the graph's (page-locked) arrays, after any edges parsed
                // sequentially before the chunked part
                g.eu.reserve(ne); g.ev.reserve(ne); g.elat.reserve(ne); g.ejitter.reserve(ne); g.eloss.reserve(ne);
                g.eu.assign(eo.eu.begin(), eo.eu.end());
                g.ev.assign(eo.ev.begin(), eo.ev.end());
                g.elat.assign(eo.lat.begin(), eo.lat.end());
                g.ejitter.assign(eo.jit.begin(), eo.jit.end());
                g.eloss.assign(eo.loss.begin(), eo.loss.end());
                for (auto& o : outs) {
                    g.eu.insert(g.eu.end(), o.eu.begin(), o.eu.end());
                    g.ev.insert(g.ev.end(), o.ev.begin(), o.ev.end());
                    g.elat.insert(g.elat.end(), o.lat.begin(), o.lat.end());
                    g.ejitter.insert(g.ejitter.end(), o.jit.begin(), o.jit.end());
                    g.eloss.insert(g.eloss.end(), o.loss.begin(), o.loss.end());
                }
                eo = EdgeOut();
                done = true;
                chunked = true;
            }
        }
        if (!done) {
            P.run(p, end, false, nullptr);
            if (P.failed) return false;
        }
    }
    if (!P.graph_seen) { err = "no <graph> element"; return false; }
    if (!chunked) {
        g.eu.assign(eo.eu.begin(), eo.eu.end());
        g.ev.assign(eo.ev.begin(), eo.ev.end());
        g.elat.assign(eo.lat.begin(), eo.lat.end());
        g.ejitter = std::move(eo.jit);
        g.eloss.assign(eo.loss.begin(), eo.loss.end());
    }
    g.E = (int64_t)g.eu.size();
    g.vid.resize((size_t)g.V);
    for (int32_t v = 0; v < g.V; v++) g.vid[(size_t)v] = ids.keys[(size_t)v].str();
    return true;
}

bool graphml_load_file(const char* path, HostGraph& g, std::string& err) {
    FILE* f = fopen(path, "rb");
    if (!f) {
        err = std::string("fopen failed: ") + strerror(errno);
        return false;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0) { fclose(f); err = "ftell failed"; return false; }
    std::unique_ptr<char[]> buf(new char[(size_t)n + 1]);
    size_t got = n ? fread(buf.get(), 1, (size_t)n, f) : 0;
    fclose(f);
    if (got != (size_t)n) { err = "short read"; return false; }
    buf[(size_t)n] = 0;
    return graphml_parse(buf.get(), (size_t)n, g, err);
}

static void xml_escape(std::string& out, const std::string& s) {
    for (char c : s) {
        switch (c) {
            case '<': out += "&lt;"; break;
            case '>': out += "&gt;"; break;
            case '&': out += "&amp;"; break;
            case '"': out += "&quot;"; break;
            default: out.push_back(c);
        }
    }
}

// shortest decimal that reads back to the same double (std::to_chars round trip)
static void put_num(std::string& out, double x) {
    char num[64];
    const auto r = std::to_chars(num, num + sizeof num, x);
    out.append(num, r.ptr);
}

// Same key schema as the bundled resource/*.graphml.xml files (d0..d9).  Nodes and edges are
// formatted in parallel chunks and written in order.
bool graphml_write_file(const HostGraph& g, const char* path) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    std::string head =
        "<?xml version=\"1.0\" encoding=\"utf-8\"?><graphml xmlns=\"http://graphml.graphdrawing.org/xmlns\">\n"
        "  <key attr.name=\"packetloss\" attr.type=\"double\" for=\"edge\" id=\"d9\" />\n"
        "  <key attr.name=\"jitter\" attr.type=\"double\" for=\"edge\" id=\"d8\" />\n"
        "  <key attr.name=\"latency\" attr.type=\"double\" for=\"edge\" id=\"d7\" />\n"
        "  <key attr.name=\"type\" attr.type=\"string\" for=\"node\" id=\"d5\" />\n"
        "  <key attr.name=\"bandwidthup\" attr.type=\"int\" for=\"node\" id=\"d4\" />\n"
        "  <key attr.name=\"bandwidthdown\" attr.type=\"int\" for=\"node\" id=\"d3\" />\n"
        "  <key attr.name=\"geocode\" attr.type=\"string\" for=\"node\" id=\"d2\" />\n"
        "  <key attr.name=\"ip\" attr.type=\"string\" for=\"node\" id=\"d1\" />\n"
        "  <key attr.name=\"packetloss\" attr.type=\"double\" for=\"node\" id=\"d0\" />\n";
    head += g.directed ? "  <graph edgedefault=\"directed\">\n" : "  <graph edgedefault=\"undirected\">\n";
    bool ok = fwrite(head.data(), 1, head.size(), f) == head.size();
    auto node = [&](std::string& out, int64_t v) {
        out += "    <node id=\"";
        xml_escape(out, g.vid[(size_t)v]);
        out += "\">\n      <data key=\"d0\">"; put_num(out, g.vloss[(size_t)v]);
        out += "</data>\n      <data key=\"d1\">"; xml_escape(out, g.vip[(size_t)v]);
        out += "</data>\n      <data key=\"d2\">"; xml_escape(out, g.vgeo[(size_t)v]);
        out += "</data>\n      <data key=\"d3\">"; put_num(out, g.vbwdown[(size_t)v]);
        out += "</data>\n      <data key=\"d4\">"; put_num(out, g.vbwup[(size_t)v]);
        out += "</data>\n      <data key=\"d5\">"; xml_escape(out, g.vtype[(size_t)v]);
        out += "</data>\n    </node>\n";
    };
    auto edge = [&](std::string& out, int64_t e) {
        out += "    <edge source=\"";
        xml_escape(out, g.vid[(size_t)g.eu[(size_t)e]]);
        out += "\" target=\"";
        xml_escape(out, g.vid[(size_t)g.ev[(size_t)e]]);
        out += "\">\n      <data key=\"d7\">"; put_num(out, g.elat[(size_t)e]);
        out += "</data>\n      <data key=\"d8\">"; put_num(out, g.ejitter[(size_t)e]);
        out += "</data>\n      <data key=\"d9\">"; put_num(out, g.eloss[(size_t)e]);
        out += "</data>\n    </edge>\n";
    };
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t kBlock = 1 << 16;  // elements per formatted block
    auto emit = [&](int64_t n, const std::function<void(std::string&, int64_t)>& fmt) {
        for (int64_t b0 = 0; b0 < n && ok; b0 += kBlock * nt) {
            std::vector<std::string> bufs(nt);
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nt; t++)
                th.emplace_back([&, t]() {
                    const int64_t lo = b0 + kBlock * t, hi = std::min(n, lo + kBlock);
                    for (int64_t i = lo; i < hi; i++) fmt(bufs[t], i);
                });
            for (auto& x : th) x.join();
            for (auto& b : bufs) ok = ok && fwrite(b.data(), 1, b.size(), f) == b.size();
        }
    };
    emit(g.V, node);
    emit(g.E, edge);
    const char* tail = "  </graph>\n</graphml>\n";
    ok = ok && fwrite(tail, 1, strlen(tail), f) == strlen(tail);
    return (fclose(f) == 0) && ok;
}

// ------------------------------------------------------------------------------------------
// Synthetic power-law Internet topology (BASELINE.json config 4; SURVEY.md 8(d) "C4").
// n_routers routers "pop-k" + n_poi points of interest "poi-k".  Edges, in this order:
//   * a random spanning path over the routers (connectivity),
//   * Chung-Lu router edges, endpoint weight ~ rank^-alpha (ranks randomly permuted over the
//     routers), deduplicated: no self loops, no parallel edges,
//   * one uplink per poi to a uniform router (latency 5.0, as tools/topology/generate-topology.py:54),
//   * one self loop per poi (the source is always one of its own targets).
// Router-edge latency ~ U[1,100) full-mantissa f64 (U{1..100} with integer_latency), edge
// packetloss ~ U[0,0.01), poi packetloss ~ U[0,0.05).  Total edges == n_edges exactly.
// ------------------------------------------------------------------------------------------
bool synth_graph(const SynthParams& p, HostGraph& g, std::string& err) {
    g = HostGraph();
    const int64_t R = p.n_routers, P = p.n_poi;
    if (R < 2 || P < 1) { err = "need >= 2 routers and >= 1 poi"; return false; }
    const int64_t n_cl = p.n_edges - (R - 1) - 2 * P;
    if (n_cl < 0) { err = "n_edges too small"; return false; }
    if ((double)n_cl > 0.45 * (double)R * (double)(R - 1)) { err = "n_edges too large"; return false; }
    SplitMix rng(p.seed);
    g.V = (int32_t)(R + P);
    g.directed = false;
    static const char* kGeo[] = {"US", "DE", "FR", "GB", "NL", "CA", "SE", "RU",
                                 "JP", "BR", "IN", "AU", "CH", "IT", "ES", "PL"};
    g.vid.resize((size_t)g.V);
    g.vtype.resize((size_t)g.V);
    g.vip.assign((size_t)g.V, "0.0.0.0");
    g.vgeo.resize((size_t)g.V);
    g.vbwup.resize((size_t)g.V);
    g.vbwdown.resize((size_t)g.V);
    g.vloss.resize((size_t)g.V);
    for (int64_t r = 0; r < R; r++) {
        g.vid[(size_t)r] = "pop-" + std::to_string(r);
        g.vtype[(size_t)r] = "pop";
        g.vgeo[(size_t)r] = kGeo[r % 16];
        g.vbwup[(size_t)r] = 0;
        g.vbwdown[(size_t)r] = 0;
        g.vloss[(size_t)r] = 0.0;
    }
    for (int64_t k = 0; k < P; k++) {
        size_t v = (size_t)(R + k);
        g.vid[v] = "poi-" + std::to_string(k);
        // a unique address per poi (tools/topology/generate-topology.py gives relay and server
        // poi their real IPs, :73,84): lets a workload pin one host to every poi by ipHint
        {
            const uint64_t a = (uint64_t)k + 1;
            g.vip[v] = "10." + std::to_string((a >> 16) & 255) + "." + std::to_string((a >> 8) & 255) +
                       "." + std::to_string(a & 255);
        }
        uint64_t t = rng.below(100);
        g.vtype[v] = t < 94 ? "client" : (t < 99 ? "relay" : "server");
        g.vgeo[v] = kGeo[rng.below(16)];
        g.vbwup[v] = (double)(1024 * (1 + rng.below(64)));
        g.vbwdown[v] = (double)(1024 * (1 + rng.below(64)));
        g.vloss[v] = 0.05 * rng.uniform();
    }
    // open-addressing set of router pairs (key = min*R + max + 1, 0 = empty)
    uint64_t cap = 1;
    while (cap < (uint64_t)(2.5 * (double)(n_cl + R))) cap <<= 1;
    std::vector<uint64_t> table(cap, 0);
    auto insert = [&](int64_t a, int64_t b) -> bool {
        if (a > b) std::swap(a, b);
        uint64_t key = (uint64_t)a * (uint64_t)R + (uint64_t)b + 1;
        uint64_t h = key * 0x9E3779B97F4A7C15ull;
        uint64_t i = (h >> 17) & (cap - 1);
        for (;;) {
            if (table[i] == 0) { table[i] = key; return true; }
            if (table[i] == key) return false;
            i = (i + 1) & (cap - 1);
        }
    };
    auto draw_lat = [&]() -> double {
        if (p.integer_latency) return (double)(1 + rng.below(100));
        return 1.0 + 99.0 * rng.uniform();
    };
    g.eu.reserve((size_t)p.n_edges);
    g.ev.reserve((size_t)p.n_edges);
    g.elat.reserve((size_t)p.n_edges);
    g.eloss.reserve((size_t)p.n_edges);
    // spanning path
    std::vector<int32_t> perm((size_t)R);
    for (int64_t i = 0; i < R; i++) perm[(size_t)i] = (int32_t)i;
    for (int64_t i = R - 1; i > 0; i--) std::swap(perm[(size_t)i], perm[(size_t)rng.below((uint64_t)i + 1)]);
    for (int64_t i = 0; i + 1 < R; i++) {
        insert(perm[(size_t)i], perm[(size_t)i + 1]);
        g.eu.push_back(perm[(size_t)i]);
        g.ev.push_back(perm[(size_t)i + 1]);
        g.elat.push_back(draw_lat());
        g.eloss.push_back(0.01 * rng.uniform());
    }
    // Chung-Lu: weights rank^-alpha, ranks randomly permuted; Vose alias table
    std::vector<int32_t> rank((size_t)R);
    for (int64_t i = 0; i < R; i++) rank[(size_t)i] = (int32_t)i;
    for (int64_t i = R - 1; i > 0; i--) std::swap(rank[(size_t)i], rank[(size_t)rng.below((uint64_t)i + 1)]);
    std::vector<double> prob((size_t)R);
    double W = 0;
    for (int64_t i = 0; i < R; i++) {
        prob[(size_t)i] = pow((double)(rank[(size_t)i] + 1), -p.alpha);
        W += prob[(size_t)i];
    }
    std::vector<int32_t> alias((size_t)R, 0);
    {
        std::vector<int32_t> small, large;
        for (int64_t i = 0; i < R; i++) {
            prob[(size_t)i] = prob[(size_t)i] * (double)R / W;
            (prob[(size_t)i] < 1.0 ? small : large).push_back((int32_t)i);
        }
        while (!small.empty() && !large.empty()) {
            int32_t s = small.back(); small.pop_back();
            int32_t l = large.back(); large.pop_back();
            alias[(size_t)s] = l;
            prob[(size_t)l] = (prob[(size_t)l] + prob[(size_t)s]) - 1.0;
            (prob[(size_t)l] < 1.0 ? small : large).push_back(l);
        }
        for (int32_t l : large) prob[(size_t)l] = 1.0;
        for (int32_t s : small) prob[(size_t)s] = 1.0;
    }
    auto sample = [&]() -> int64_t {
        int64_t i = (int64_t)rng.below((uint64_t)R);
        return rng.uniform() < prob[(size_t)i] ? i : alias[(size_t)i];
    };
    int64_t made = 0;
    uint64_t guard = 0;
    while (made < n_cl) {
        if (++guard > (uint64_t)n_cl * 200 + 1000000) { err = "Chung-Lu sampling did not converge"; return false; }
        int64_t a = sample(), b = sample();
        if (a == b) continue;
        if (!insert(a, b)) continue;
        g.eu.push_back((int32_t)a);
        g.ev.push_back((int32_t)b);
        g.elat.push_back(draw_lat());
        g.eloss.push_back(0.01 * rng.uniform());
        made++;
    }
    // poi uplinks then self loops
    for (int64_t k = 0; k < P; k++) {
        g.eu.push_back((int32_t)(R + k));
        g.ev.push_back((int32_t)rng.below((uint64_t)R));
        g.elat.push_back(5.0);
        g.eloss.push_back(0.0);
    }
    for (int64_t k = 0; k < P; k++) {
        g.eu.push_back((int32_t)(R + k));
        g.ev.push_back((int32_t)(R + k));
        g.elat.push_back(p.integer_latency ? (double)(1 + rng.below(10)) : 1.0 + 9.0 * rng.uniform());
        g.eloss.push_back(0.01 * rng.uniform());
    }
    if (p.directed) {
        // every non-loop edge also the other way, with its own draws (uplinks stay 5.0): the
        // spanning path in both directions keeps the graph strongly connected
        g.directed = true;
        const size_t n = g.eu.size();
        for (size_t e = 0; e < n; e++) {
            if (g.eu[e] == g.ev[e]) continue;
            const bool uplink = g.eu[e] >= (int32_t)R;
            g.eu.push_back(g.ev[e]);
            g.ev.push_back(g.eu[e]);
            g.elat.push_back(uplink ? 5.0 : draw_lat());
            g.eloss.push_back(uplink ? 0.0 : 0.01 * rng.uniform());
        }
    }
    g.E = (int64_t)g.eu.size();
    g.ejitter.assign((size_t)g.E, 0.0);
    return true;
}

void AttachIndex::build(const HostGraph& g) {
    all.clear(); byType.clear(); byCode.clear(); byTypeCode.clear(); byIP.clear();
    ip.assign((size_t)g.V, 0xFFFFFFFFu);
    usable.assign((size_t)g.V, 0);
    auto lower = [](const std::string& s) {
        std::string o(s);
        for (auto& c : o) if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
        return o;
    };
    for (int32_t v = 0; v < g.V; v++) {
        if (g.vid[(size_t)v].find("poi") == std::string::npos) continue;  // shd-topology.c:974
        uint32_t a = string_to_ip(g.vip[(size_t)v].c_str());
        ip[(size_t)v] = a;
        usable[(size_t)v] = (a != 0xFFFFFFFFu && a != 0u);
        all.push_back(v);
        std::string t = lower(g.vtype[(size_t)v]), c = lower(g.vgeo[(size_t)v]);
        byType[t].push_back(v);
        byCode[c].push_back(v);
        byTypeCode[t + '\x01' + c].push_back(v);
        byIP[a].push_back(v);
    }
    built = true;
}

}  // namespace shdtopo
