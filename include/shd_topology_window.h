/*
 * shd_topology_window.h -- the engine-side window adapter of libshdtopo.so:
 * worker_schedulePacket (src/engine/shd-worker.c:332-370) deferred to the scheduler's window
 * barrier and run as one GPU batch (topology_routePacketBatch).
 *
 * Shadow integration:
 *   at emit   -- shd-worker.c:345-369 becomes  topowindow_emit(w, src, dst, payloadLength,
 *                host_getRandom(srcHost), worker_getCurrentTime(), packet);
 *                it records the packet with the sender stream's state BEFORE the reference's
 *                one draw and advances that stream by the draw, so every later
 *                consumer of the host stream sees the reference sequence;
 *   barrier   -- multi-threaded: at shd-slave.c:415 (all workers parked at processingLatch)
 *                topowindow_flush(w, slave_getMinTimeJump(slave), 1, deliver, ctx);
 *                deliver() schedules the PacketArrivedEvent at out->time (worker_scheduleEvent
 *                without its own clamp: the clamp of shd-worker.c:310-324 is applied here);
 *   serial    -- the reference runs one unbounded window (shd-master.c:220-224).  Packets are
 *                still safe to defer for topowindow_serial_window_ns() ns: an arrival is at
 *                least emit + minimum latency >= the window end.  slave_runSerial flushes with
 *                multiThreaded = 0 (no clamp, as the reference in serial mode) whenever the next
 *                event reaches the window end.
 *
 * Ordering: packets are routed in the order topowindow_emit recorded them (one lock: the
 * real-time interleaving of the worker threads, which is what the reference's lazy cache sees;
 * inside one worker, its emission order).  Arrival events with equal times are scheduled in
 * that order (receiver queue sequence numbers, shd-event-queue.c:44-54).
 *
 * The sender's pre-draw state is the first field of Shadow's Random (struct _Random
 * { guint seedState; guint initialSeed; }, src/utility/shd-random.c:13-16); the draw itself goes
 * through random_nextDouble (imported from the executable, like the Part 1 imports).
 */
#ifndef SHD_TOPOLOGY_WINDOW_H_
#define SHD_TOPOLOGY_WINDOW_H_

#include "shd_topology_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _TopoWindow TopoWindow;

/* deliver(ctx, packet, delivered, time): one call per recorded packet at flush, in order;
 * delivered = 0 for a dropped packet (PDS_INET_DROPPED, no event), time = arrival ns */
typedef void (*TopoWindowDeliver)(void* ctx, void* packet, int delivered, uint64_t time);

TopoWindow* topowindow_new(Topology* top);
void topowindow_free(TopoWindow* w);

/* record one packet of the current window (thread-safe); returns its index in the window, or -1
 * if an address is not attached (the reference's getters return -1.0 and the packet is lost:
 * PDS_INET_DROPPED, the draw is still taken).  payloadLength 0 = control packet (never dropped). */
int64_t topowindow_emit(TopoWindow* w, Address* src, Address* dst, uint32_t payloadLength,
                        Random* senderRandom, uint64_t now, void* packet);
/* same, with the caller's own capture of the pre-draw state (the caller advances its stream) */
int64_t topowindow_emit_state(TopoWindow* w, uint32_t srcIP, uint32_t dstIP,
                              uint32_t payloadLength, uint32_t preDrawState, uint64_t now,
                              void* packet);

/* packets recorded since the last flush */
int64_t topowindow_pending(TopoWindow* w);

/* route every recorded packet in one batch on the GPU, then deliver them in order and clear the
 * window.  jumpNs / multiThreaded: the inter-host clamp of shd-worker.c:310-324 (0 = serial).
 * Vertices are resolved at emit: a packet whose sender or receiver was detached since is still
 * routed while its vertex keeps another host (the table's columns), else delivered 0 (dropped).
 * Returns 0, or a negative error of the batch -- then nothing is delivered and the packets stay
 * recorded (in order, before any emitted since) for the next flush. */
int topowindow_flush(TopoWindow* w, uint64_t jumpNs, int multiThreaded, TopoWindowDeliver deliver,
                     void* ctx);

/* multi-threaded window (the reference's runahead, shd-master.c:98-124): (u64) minimum latency
 * in whole ms -- here the eager global minimum (topology_getMinimumLatency) -- 10 ms if unknown,
 * raised to runaheadNs (--runahead).  Inter-host arrivals are clamped to now + this. */
uint64_t topowindow_jump_ns(Topology* top, uint64_t runaheadNs);
/* serial-mode window: the longest window whose packets can all be routed at its end without
 * changing any arrival time: floor(minimum latency x 1e6) ns (an arrival is emit + ceil(latency
 * x 1e6) >= window start + that), at least 1 ns.  No clamp in serial mode, as the reference. */
uint64_t topowindow_serial_window_ns(Topology* top);

#ifdef __cplusplus
}
#endif
#endif /* SHD_TOPOLOGY_WINDOW_H_ */
