// topo_window.cpp -- the engine-side window adapter (include/shd_topology_window.h, SURVEY.md
// 8(f)#3): worker_schedulePacket (src/engine/shd-worker.c:332-370) recorded at emit and routed
// as one GPU batch at the scheduler's window barrier (shd-slave.c:415-461).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/shd_topology_window.h"

extern "C" {
__attribute__((weak)) uint32_t address_toNetworkIP(Address* address);
__attribute__((weak)) double random_nextDouble(Random* random);
}

// One recorded packet: its vertices are resolved at emit, when the reference routed it
// (shd-worker.c:345-369), so a host detached before the flush does not lose its packets.
struct WinPacket {
    int32_t srcV, dstV;
    uint32_t payloadLength, rngState;
    uint64_t now;
    void* packet;
};

struct _TopoWindow {
    Topology* top = nullptr;
    std::mutex mu;  // worker threads emit concurrently; the window keeps their real-time order
    std::vector<WinPacket> in;
    std::vector<TopoPacketOut> out;
};

extern "C" {

TopoWindow* topowindow_new(Topology* top) {
    if (!top) return nullptr;
    TopoWindow* w = new TopoWindow();
    w->top = top;
    shdtopo_window_hold(top, +1);
    return w;
}

void topowindow_free(TopoWindow* w) {
    if (!w) return;
    shdtopo_window_hold(w->top, -1);
    shdtopo_window_release(w->top);
    delete w;
}

int64_t topowindow_emit_state(TopoWindow* w, uint32_t srcIP, uint32_t dstIP,
                              uint32_t payloadLength, uint32_t preDrawState, uint64_t now,
                              void* packet) {
    if (!w) return -1;
    // the reference's getters return -1.0 for an address the topology does not know (the
    // packet is then dropped unless a control packet): not routed here, the caller drops it
    const int32_t sv = shdtopo_vertex_of_ip(w->top, srcIP), dv = shdtopo_vertex_of_ip(w->top, dstIP);
    if (sv < 0 || dv < 0) return -1;
    std::lock_guard<std::mutex> lk(w->mu);
    w->in.push_back(WinPacket{sv, dv, payloadLength, preDrawState, now, packet});
    return (int64_t)w->in.size() - 1;
}

int64_t topowindow_emit(TopoWindow* w, Address* src, Address* dst, uint32_t payloadLength,
                        Random* senderRandom, uint64_t now, void* packet) {
    if (!w || !src || !dst || !senderRandom || !address_toNetworkIP || !random_nextDouble)
        return -1;
    // Shadow's Random is { guint seedState; guint initialSeed; } (shd-random.c:13-16): the state
    // before the reference's one draw (shd-worker.c:353-354), then that draw on the stream
    uint32_t pre;
    memcpy(&pre, (const void*)senderRandom, sizeof pre);
    (void)random_nextDouble(senderRandom);
    return topowindow_emit_state(w, address_toNetworkIP(src), address_toNetworkIP(dst),
                                 payloadLength, pre, now, packet);
}

int64_t topowindow_pending(TopoWindow* w) {
    if (!w) return -1;
    std::lock_guard<std::mutex> lk(w->mu);
    return (int64_t)w->in.size();
}

int topowindow_flush(TopoWindow* w, uint64_t jumpNs, int multiThreaded, TopoWindowDeliver deliver,
                     void* ctx) {
    if (!w) return -1;
    std::vector<WinPacket> in;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        in.swap(w->in);
    }
    if (in.empty()) {
        shdtopo_window_release(w->top);
        return 0;
    }
    const size_t n = in.size();
    std::vector<int32_t> sv(n), dv(n);
    std::vector<uint32_t> pay(n), st(n);
    std::vector<uint64_t> now(n);
    for (size_t i = 0; i < n; i++) {
        sv[i] = in[i].srcV;
        dv[i] = in[i].dstV;
        pay[i] = in[i].payloadLength;
        st[i] = in[i].rngState;
        now[i] = in[i].now;
    }
    w->out.resize(n);
    // a vertex detached during the window is still a column (shdtopo_window_hold): its packets
    // are routed as at emit; only a packet whose vertex left before an earlier flush comes back
    // undelivered
    const int r = shdtopo_route_batch_vertices(w->top, sv.data(), dv.data(), pay.data(), st.data(),
                                               now.data(), n, jumpNs, multiThreaded, w->out.data());
    if (r < 0) {
        // nothing was routed: the window is put back in front of what was emitted meanwhile, so
        // a later flush routes every packet in emission order
        std::lock_guard<std::mutex> lk(w->mu);
        in.insert(in.end(), w->in.begin(), w->in.end());
        w->in.swap(in);
        return r;
    }
    // the window's packets are routed: vertices detached during it may leave the table now
    shdtopo_window_release(w->top);
    if (deliver)
        for (size_t i = 0; i < n; i++)
            deliver(ctx, in[i].packet, w->out[i].delivered, w->out[i].time);
    return 0;
}

uint64_t topowindow_jump_ns(Topology* top, uint64_t runaheadNs) {
    const double m = topology_getMinimumLatency(top);
    uint64_t jump = m > 0 ? ((uint64_t)m) * 1000000ull : 0;  // shd-master.c:118
    if (jump == 0) jump = 10ull * 1000000ull;                 // shd-master.c:103
    if (runaheadNs > 0 && jump < runaheadNs) jump = runaheadNs;  // :106-108
    return jump;
}

uint64_t topowindow_serial_window_ns(Topology* top) {
    const double m = topology_getMinimumLatency(top);
    const double ns = m > 0 ? std::floor(m * 1000000.0) : 0.0;
    return ns >= 1.0 ? (uint64_t)ns : 1ull;
}

}  // extern "C"
