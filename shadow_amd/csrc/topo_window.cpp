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

struct _TopoWindow {
    Topology* top = nullptr;
    std::mutex mu;  // worker threads emit concurrently; the window keeps their real-time order
    std::vector<TopoPacketIn> in;
    std::vector<void*> packets;
    std::vector<TopoPacketOut> out;
};

extern "C" {

TopoWindow* topowindow_new(Topology* top) {
    if (!top) return nullptr;
    TopoWindow* w = new TopoWindow();
    w->top = top;
    return w;
}

void topowindow_free(TopoWindow* w) { delete w; }

int64_t topowindow_emit_state(TopoWindow* w, uint32_t srcIP, uint32_t dstIP,
                              uint32_t payloadLength, uint32_t preDrawState, uint64_t now,
                              void* packet) {
    if (!w) return -1;
    // the reference's getters return -1.0 for an address the topology does not know (the
    // packet is then dropped unless a control packet): not routed here, the caller drops it
    if (shdtopo_vertex_of_ip(w->top, srcIP) < 0 || shdtopo_vertex_of_ip(w->top, dstIP) < 0)
        return -1;
    TopoPacketIn p;
    p.srcIP = srcIP;
    p.dstIP = dstIP;
    p.payloadLength = payloadLength;
    p.rngState = preDrawState;
    p.now = now;
    std::lock_guard<std::mutex> lk(w->mu);
    w->in.push_back(p);
    w->packets.push_back(packet);
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
    std::vector<TopoPacketIn> in;
    std::vector<void*> packets;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        in.swap(w->in);
        packets.swap(w->packets);
    }
    if (in.empty()) return 0;
    w->out.resize(in.size());
    const int r = topology_routePacketBatch(w->top, in.data(), w->out.data(), in.size(), jumpNs,
                                            multiThreaded);
    if (r) return r;
    if (deliver)
        for (size_t i = 0; i < in.size(); i++)
            deliver(ctx, packets[i], w->out[i].delivered, w->out[i].time);
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
