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
#include <fstream>
#include <sstream>

#include "topo_internal.h"

namespace shdtopo {

uint32_t string_to_ip(const char* s) {
    if (!s) return 0xFFFFFFFFu;  // INADDR_NONE
    struct in_addr a;
    if (inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return 0xFFFFFFFFu;
}

namespace {

struct Key {
    std::string name, type, forwhat, def;
    bool has_default = false;
    bool numeric() const {
        return type == "double" || type == "float" || type == "int" || type == "long" ||
               type == "integer";
    }
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

std::string decode_entities(const char* b, const char* e) {
    std::string out;
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
    return out;
}

struct Tag {
    std::string name;  // local name (namespace prefix stripped)
    bool closing = false, selfclose = false;
    std::vector<std::pair<std::string, std::string>> attrs;
    const char* attr(const char* k) const {
        for (auto& a : attrs)
            if (a.first == k) return a.second.c_str();
        return nullptr;
    }
};

// parse one tag starting at p ('<'), return pointer past '>' or nullptr
const char* parse_tag(const char* p, const char* end, Tag& t) {
    t.attrs.clear();
    t.closing = t.selfclose = false;
    ++p;
    if (p < end && *p == '/') { t.closing = true; ++p; }
    const char* nb = p;
    while (p < end && !is_space(*p) && *p != '>' && *p != '/') ++p;
    const char* colon = (const char*)memchr(nb, ':', (size_t)(p - nb));
    t.name.assign(colon ? colon + 1 : nb, p);
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
        std::string k(kb, p);
        while (p < end && is_space(*p)) ++p;
        if (p < end && *p == '=') {
            ++p;
            while (p < end && is_space(*p)) ++p;
            if (p >= end) return nullptr;
            char q = *p;
            if (q != '"' && q != '\'') return nullptr;
            ++p;
            const char* vb = p;
            const char* ve = (const char*)memchr(p, q, (size_t)(end - p));
            if (!ve) return nullptr;
            t.attrs.emplace_back(k, decode_entities(vb, ve));
            p = ve + 1;
        } else {
            t.attrs.emplace_back(k, std::string());
        }
    }
}

double parse_numeric(const std::string& s) {
    const char* c = s.c_str();
    while (*c && is_space(*c)) ++c;
    if (!*c) return NAN;
    char* endp = nullptr;
    double v = strtod(c, &endp);
    if (endp == c) return NAN;
    return v;
}

}  // namespace

bool graphml_parse(const char* buf, size_t len, HostGraph& g, std::string& err) {
    g = HostGraph();
    const char* p = buf;
    const char* end = buf + len;
    std::unordered_map<std::string, Key> keys;
    std::unordered_map<std::string, int32_t> node_index;
    node_index.reserve(1 << 16);
    Tag t;
    enum { NONE, IN_KEY, IN_NODE, IN_EDGE } ctx = NONE;
    std::string cur_key_id;
    Key cur_key;
    bool in_default = false, in_data = false;
    std::string data_key, text;
    // per-element collected data
    std::vector<std::pair<std::string, std::string>> elem_data;
    int32_t cur_vertex = -1;
    bool graph_seen = false;

    // attribute schema resolved lazily per key id
    auto vertex_of = [&](const std::string& id) -> int32_t {
        auto it = node_index.find(id);
        if (it != node_index.end()) return it->second;
        int32_t v = g.V++;
        node_index.emplace(id, v);
        g.vid.push_back(id);
        return v;
    };

    struct EdgePending { int32_t u, v; };
    std::vector<std::vector<std::pair<std::string, std::string>>> vdata;  // per vertex raw data
    std::vector<std::vector<std::pair<std::string, std::string>>> edata;

    while (p < end) {
        if (*p != '<') {
            const char* q = (const char*)memchr(p, '<', (size_t)(end - p));
            if (!q) q = end;
            if (in_data || in_default) text.append(p, q);
            p = q;
            continue;
        }
        if (end - p >= 4 && !memcmp(p, "<!--", 4)) {
            const char* q = strstr(p + 4, "-->");
            if (!q) { err = "unterminated comment"; return false; }
            p = q + 3;
            continue;
        }
        if (end - p >= 9 && !memcmp(p, "<![CDATA[", 9)) {
            const char* q = strstr(p + 9, "]]>");
            if (!q) { err = "unterminated CDATA"; return false; }
            if (in_data || in_default) {
                // CDATA text is literal: escape '&' so decode_entities leaves it intact
                for (const char* c = p + 9; c < q; ++c) {
                    if (*c == '&') text += "&amp;"; else text.push_back(*c);
                }
            }
            p = q + 3;
            continue;
        }
        if (end - p >= 2 && (p[1] == '?' || p[1] == '!')) {
            const char* q = (const char*)memchr(p, '>', (size_t)(end - p));
            if (!q) { err = "unterminated declaration"; return false; }
            p = q + 1;
            continue;
        }
        const char* nx = parse_tag(p, end, t);
        if (!nx) { err = "malformed tag"; return false; }
        p = nx;
        const std::string& nm = t.name;
        if (!t.closing) {
            if (nm == "key") {
                cur_key = Key();
                const char* id = t.attr("id");
                cur_key_id = id ? id : "";
                const char* an = t.attr("attr.name");
                cur_key.name = an ? an : cur_key_id;
                const char* at = t.attr("attr.type");
                cur_key.type = at ? at : "string";
                const char* fo = t.attr("for");
                cur_key.forwhat = fo ? fo : "all";
                if (t.selfclose) keys[cur_key_id] = cur_key;
                else ctx = IN_KEY;
            } else if (nm == "default" && ctx == IN_KEY) {
                in_default = !t.selfclose;
                text.clear();
                if (t.selfclose) { cur_key.has_default = true; cur_key.def.clear(); }
            } else if (nm == "graph") {
                const char* ed = t.attr("edgedefault");
                // GraphML: edgedefault is required; igraph treats a missing one as directed
                g.directed = !(ed && !strcmp(ed, "undirected"));
                graph_seen = true;
            } else if (nm == "node") {
                const char* id = t.attr("id");
                if (!id) { err = "node without id"; return false; }
                // first appearance creates the vertex; data of a re-declared id is ignored
                bool existed = node_index.count(id) != 0;
                cur_vertex = vertex_of(id);
                if (existed) cur_vertex = -1;
                if ((int32_t)vdata.size() < g.V) vdata.resize((size_t)g.V);
                elem_data.clear();
                if (t.selfclose) cur_vertex = -1;
                else ctx = IN_NODE;
            } else if (nm == "edge") {
                const char* s = t.attr("source");
                const char* d = t.attr("target");
                if (!s || !d) { err = "edge without source/target"; return false; }
                int32_t u = vertex_of(s), v = vertex_of(d);
                if ((int32_t)vdata.size() < g.V) vdata.resize((size_t)g.V);
                g.eu.push_back(u);
                g.ev.push_back(v);
                edata.emplace_back();
                elem_data.clear();
                if (!t.selfclose) ctx = IN_EDGE;
            } else if (nm == "data" && (ctx == IN_NODE || ctx == IN_EDGE)) {
                const char* k = t.attr("key");
                data_key = k ? k : "";
                text.clear();
                if (t.selfclose) elem_data.emplace_back(data_key, std::string());
                else in_data = true;
            }
        } else {
            if (nm == "key" && ctx == IN_KEY) {
                keys[cur_key_id] = cur_key;
                ctx = NONE;
            } else if (nm == "default" && in_default) {
                cur_key.def = decode_entities(text.data(), text.data() + text.size());
                cur_key.has_default = true;
                in_default = false;
            } else if (nm == "data" && in_data) {
                elem_data.emplace_back(data_key,
                                       decode_entities(text.data(), text.data() + text.size()));
                in_data = false;
            } else if (nm == "node" && ctx == IN_NODE) {
                if (cur_vertex >= 0) {
                    auto& dst = vdata[(size_t)cur_vertex];
                    for (auto& kv : elem_data) dst.push_back(std::move(kv));
                }
                ctx = NONE;
                cur_vertex = -1;
            } else if (nm == "edge" && ctx == IN_EDGE) {
                edata.back() = std::move(elem_data);
                elem_data.clear();
                ctx = NONE;
            }
        }
    }
    if (!graph_seen) { err = "no <graph> element"; return false; }
    g.E = (int64_t)g.eu.size();

    // resolve attributes by name, honouring the key's domain (vertex and edge packetloss are
    // distinct namespaces)
    auto find_key = [&](const char* name, bool for_node) -> const std::pair<const std::string, Key>* {
        for (auto& kv : keys) {
            const Key& k = kv.second;
            bool dom = k.forwhat == "all" || (for_node ? k.forwhat == "node" : k.forwhat == "edge");
            if (dom && k.name == name) return &kv;
        }
        return nullptr;
    };
    auto fill_num = [&](const char* name, bool for_node,
                        const std::vector<std::vector<std::pair<std::string, std::string>>>& data,
                        size_t n, std::vector<double>& out) {
        out.assign(n, NAN);
        auto* k = find_key(name, for_node);
        if (!k) return;
        double def = k->second.has_default ? parse_numeric(k->second.def) : NAN;
        for (size_t i = 0; i < n; i++) {
            out[i] = def;
            if (i < data.size())
                for (auto& kv : data[i])
                    if (kv.first == k->first) out[i] = parse_numeric(kv.second);
        }
    };
    auto fill_str = [&](const char* name, bool for_node,
                        const std::vector<std::vector<std::pair<std::string, std::string>>>& data,
                        size_t n, std::vector<std::string>& out) {
        out.assign(n, std::string());
        auto* k = find_key(name, for_node);
        if (!k) return;
        for (size_t i = 0; i < n; i++) {
            if (k->second.has_default) out[i] = k->second.def;
            if (i < data.size())
                for (auto& kv : data[i])
                    if (kv.first == k->first) out[i] = kv.second;
        }
    };
    vdata.resize((size_t)g.V);
    fill_str("type", true, vdata, (size_t)g.V, g.vtype);
    fill_str("ip", true, vdata, (size_t)g.V, g.vip);
    fill_str("geocode", true, vdata, (size_t)g.V, g.vgeo);
    fill_num("bandwidthup", true, vdata, (size_t)g.V, g.vbwup);
    fill_num("bandwidthdown", true, vdata, (size_t)g.V, g.vbwdown);
    fill_num("packetloss", true, vdata, (size_t)g.V, g.vloss);
    fill_num("latency", false, edata, (size_t)g.E, g.elat);
    fill_num("jitter", false, edata, (size_t)g.E, g.ejitter);
    fill_num("packetloss", false, edata, (size_t)g.E, g.eloss);
    return true;
}

bool graphml_load_file(const char* path, HostGraph& g, std::string& err) {
    FILE* f = fopen(path, "rb");
    if (!f) {
        err = std::string("fopen failed: ") + strerror(errno);
        return false;
    }
    std::string buf;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0) { fclose(f); err = "ftell failed"; return false; }
    buf.resize((size_t)n);
    size_t got = n ? fread(&buf[0], 1, (size_t)n, f) : 0;
    fclose(f);
    if (got != (size_t)n) { err = "short read"; return false; }
    return graphml_parse(buf.data(), buf.size(), g, err);
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

// Same key schema as the bundled resource/*.graphml.xml files (d0..d9).
bool graphml_write_file(const HostGraph& g, const char* path) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    std::string out;
    out.reserve(1 << 20);
    out +=
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
    out += g.directed ? "  <graph edgedefault=\"directed\">\n" : "  <graph edgedefault=\"undirected\">\n";
    char num[64];
    auto flush = [&]() {
        if (out.size() > (1u << 20)) {
            fwrite(out.data(), 1, out.size(), f);
            out.clear();
        }
    };
    for (int32_t v = 0; v < g.V; v++) {
        out += "    <node id=\"";
        xml_escape(out, g.vid[(size_t)v]);
        out += "\">\n";
        snprintf(num, sizeof num, "%.17g", g.vloss[(size_t)v]);
        out += "      <data key=\"d0\">"; out += num; out += "</data>\n";
        out += "      <data key=\"d1\">"; xml_escape(out, g.vip[(size_t)v]); out += "</data>\n";
        out += "      <data key=\"d2\">"; xml_escape(out, g.vgeo[(size_t)v]); out += "</data>\n";
        snprintf(num, sizeof num, "%.17g", g.vbwdown[(size_t)v]);
        out += "      <data key=\"d3\">"; out += num; out += "</data>\n";
        snprintf(num, sizeof num, "%.17g", g.vbwup[(size_t)v]);
        out += "      <data key=\"d4\">"; out += num; out += "</data>\n";
        out += "      <data key=\"d5\">"; xml_escape(out, g.vtype[(size_t)v]); out += "</data>\n";
        out += "    </node>\n";
        flush();
    }
    for (int64_t e = 0; e < g.E; e++) {
        out += "    <edge source=\"";
        xml_escape(out, g.vid[(size_t)g.eu[(size_t)e]]);
        out += "\" target=\"";
        xml_escape(out, g.vid[(size_t)g.ev[(size_t)e]]);
        out += "\">\n";
        snprintf(num, sizeof num, "%.17g", g.elat[(size_t)e]);
        out += "      <data key=\"d7\">"; out += num; out += "</data>\n";
        snprintf(num, sizeof num, "%.17g", g.ejitter[(size_t)e]);
        out += "      <data key=\"d8\">"; out += num; out += "</data>\n";
        snprintf(num, sizeof num, "%.17g", g.eloss[(size_t)e]);
        out += "      <data key=\"d9\">"; out += num; out += "</data>\n";
        out += "    </edge>\n";
        flush();
    }
    out += "  </graph>\n</graphml>\n";
    fwrite(out.data(), 1, out.size(), f);
    return fclose(f) == 0;
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
