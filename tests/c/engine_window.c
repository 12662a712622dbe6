/*
 * engine_window.c -- the engine-side window adapter of SURVEY.md 8(f)#3, driven through the C ABI
 * exactly as Shadow's worker would drive it, and checked against the reference's per-packet
 * sequence (src/engine/shd-worker.c:332-370) run on a twin topology.
 *
 *   reference (per packet, at emit):   rel = topology_getReliability(src, dst)
 *                                      chance = random_nextDouble(sender->random)
 *                                      if (chance <= rel || payload == 0) {
 *                                          delay = ceil(topology_getLatency(src, dst) * 1e6)
 *                                          time = max(now + delay, now + jump)   (multi-threaded)
 *                                      }
 *   adapter (at emit):                 topowindow_emit(): records {src, dst, payload, sender
 *                                      state BEFORE the draw, now}, advances the sender's Random
 *                                      by the one draw
 *   adapter (at the window barrier):   topowindow_flush() -> deliver(packet, delivered, time)
 * Multi-threaded windows (jump = the runahead, clamp on) and serial-mode windows
 * (topowindow_serial_window_ns, no clamp: shd-master.c:220-224 runs serial mode unwindowed).
 *
 * Senders also draw from their host stream between packets (Shadow's process emulation uses
 * the host Random), so the captured state is not a simple function of the window start.
 * Both topologies run in lazy mode: the batch must reproduce the first-rooted-wins orientation
 * and the running-minimum trajectory (worker_updateMinTimeJump) of the per-packet getters.
 *
 * usage: engine_window [windows packets_per_window [serial]]   exit 0 = identical, 1 = mismatch
 * Test infrastructure: links libshdtopo.so + libshdtopo_shim.so only (no oracle).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/shd_topology_abi.h"
#include "../../include/shd_topology_window.h"

/* libshdtopo_shim.so (restatements of Shadow's Address / Random) */
Address* shim_address_new(uint32_t networkIP);
Random* random_new(unsigned int seed);
int random_nextInt(Random* r);
double random_nextDouble(Random* r);
unsigned int shim_random_state(Random* r);

typedef struct {
    Address* addr;
    uint32_t ip;
    Random* rngRef; /* the host stream as the reference consumes it */
    Random* rngBat; /* the same stream under the adapter */
} Host;

static uint64_t lcg = 0x9E3779B97F4A7C15ull; /* workload choices, independent of host streams */
static uint32_t pick(uint32_t n) {
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)((lcg >> 33) % n);
}

typedef struct {
    uint8_t* dl;
    uint64_t* t;
    long calls;
} Got;

static void deliver(void* ctx, void* packet, int delivered, uint64_t time) {
    Got* g = (Got*)ctx;
    const long k = (long)(intptr_t)packet;
    g->dl[k] = (uint8_t)delivered;
    g->t[k] = time;
    g->calls++;
}

static Topology* make_topology(void) {
    ShdSynthParams p = {20261016ull, 3000, 150, 30000, 0, 1.0 / 1.1};
    Topology* t = shdtopo_new_synthetic(&p);
    if (t) shdtopo_set_option(t, "lazy", 1);
    return t;
}

int main(int argc, char** argv) {
    const int windows = argc > 1 ? atoi(argv[1]) : 4;
    const int perWindow = argc > 2 ? atoi(argv[2]) : 20000;
    const int serial = argc > 3 ? atoi(argv[3]) : 0;
    const int nHosts = 400;
    Topology* ref = make_topology();
    Topology* bat = make_topology();
    if (!ref || !bat) {
        fprintf(stderr, "topology_new failed\n");
        return 2;
    }
    /* Shadow's seed chain: master (--seed 1) -> slave seed -> per-host nodeSeed */
    Random* master = random_new(1);
    Random* slave = random_new((unsigned)random_nextInt(master));
    Host* h = (Host*)calloc((size_t)nHosts, sizeof(Host));
    static const char* types[] = {"client", "relay", "server"};
    for (int k = 0; k < nHosts; k++) {
        const unsigned seed = (unsigned)random_nextInt(slave);
        h[k].ip = (11u) | (0u << 8) | ((uint32_t)(k >> 8) << 16) | ((uint32_t)((k & 255) + 1) << 24);
        h[k].addr = shim_address_new(h[k].ip);
        h[k].rngRef = random_new(seed);
        h[k].rngBat = random_new(seed);
        uint64_t bd1 = 0, bu1 = 0, bd2 = 0, bu2 = 0;
        topology_attach(ref, h[k].addr, h[k].rngRef, NULL, NULL, (char*)types[k % 3], &bd1, &bu1);
        topology_attach(bat, h[k].addr, h[k].rngBat, NULL, NULL, (char*)types[k % 3], &bd2, &bu2);
        if (bd1 != bd2 || bu1 != bu2) {
            fprintf(stderr, "attach mismatch at host %d\n", k);
            return 1;
        }
    }
    /* runahead: shd-master.c:113-124 truncates the minimum latency to whole ms */
    const double gmin = topology_getMinimumLatency(bat);
    if (topology_getMinimumLatency(ref) != gmin) return 1;
    const uint64_t jump = serial ? topowindow_serial_window_ns(bat) : topowindow_jump_ns(bat, 0);
    if (!serial && jump != (uint64_t)gmin * 1000000ull) return 1;
    TopoWindow* win = topowindow_new(bat);
    Got got;
    got.dl = (uint8_t*)calloc((size_t)perWindow, 1);
    got.t = (uint64_t*)calloc((size_t)perWindow, 8);
    uint32_t* batS = (uint32_t*)calloc((size_t)perWindow, 4);
    uint8_t* refDl = (uint8_t*)calloc((size_t)perWindow, 1);
    uint64_t* refT = (uint64_t*)calloc((size_t)perWindow, 8);
    uint32_t* refS = (uint32_t*)calloc((size_t)perWindow, 4);
    long mism = 0, delivered = 0, total = 0, reversed = 0;
    uint64_t t0 = 1000000000ull;
    for (int w = 0; w < windows; w++) {
        int n = 0;
        for (int k = 0; k < perWindow; k++) {
            const uint32_t s = pick((uint32_t)nHosts);
            uint32_t d = pick((uint32_t)nHosts - 1);
            if (d >= s) d++; /* self-destined packets never reach the topology */
            const uint32_t payload = pick(5) ? 1448u : 0u;
            const uint64_t now = t0 + pick(jump ? (uint32_t)jump : 10000000u);
            /* the sender's process draws from the host stream in between */
            for (uint32_t x = pick(3); x > 0; x--) {
                random_nextDouble(h[s].rngRef);
                random_nextDouble(h[s].rngBat);
            }
            /* ---- reference: shd-worker.c:345-369 at emit ---- */
            const double rel = topology_getReliability(ref, h[s].addr, h[d].addr);
            const double chance = random_nextDouble(h[s].rngRef);
            refDl[n] = (chance <= rel || payload == 0) ? 1 : 0;
            refT[n] = 0;
            if (refDl[n]) {
                const double lat = topology_getLatency(ref, h[s].addr, h[d].addr);
                uint64_t t = now + (uint64_t)ceil(lat * 1000000.0);
                if (!serial && t < now + jump) t = now + jump;
                if (serial && t < t0 + jump) {
                    fprintf(stderr, "serial window: arrival %llu before the window end\n",
                            (unsigned long long)t);
                    mism++;
                }
                refT[n] = t;
            }
            refS[n] = shim_random_state(h[s].rngRef);
            /* ---- adapter, emit half (the product's topowindow_emit) ---- */
            if (topowindow_emit(win, h[s].addr, h[d].addr, payload, h[s].rngBat, now,
                                (void*)(intptr_t)n) != n) {
                fprintf(stderr, "topowindow_emit failed\n");
                return 2;
            }
            batS[n] = shim_random_state(h[s].rngBat);
            n++;
        }
        /* ---- adapter, barrier half (shd-slave.c:415): one batch for the window ---- */
        got.calls = 0;
        if (topowindow_pending(win) != n ||
            topowindow_flush(win, jump, serial ? 0 : 1, deliver, &got) != 0 || got.calls != n) {
            fprintf(stderr, "topowindow_flush failed\n");
            return 2;
        }
        for (int k = 0; k < n; k++) {
            total++;
            delivered += got.dl[k];
            if (got.dl[k] != refDl[k] || got.t[k] != refT[k] || batS[k] != refS[k]) {
                if (mism < 5)
                    fprintf(stderr, "window %d packet %d: batch (%u, %llu, %u) reference (%u, %llu, %u)\n",
                            w, k, got.dl[k], (unsigned long long)got.t[k], batS[k],
                            refDl[k], (unsigned long long)refT[k], refS[k]);
                mism++;
            }
        }
        /* every host stream ends the window where the reference leaves it */
        for (int k = 0; k < nHosts; k++)
            if (shim_random_state(h[k].rngRef) != shim_random_state(h[k].rngBat)) mism++;
        /* the same lazily materialised minimum (runahead input) */
        const double m1 = shdtopo_get_lazy_minimum_latency(ref);
        const double m2 = shdtopo_get_lazy_minimum_latency(bat);
        if (m1 != m2) {
            fprintf(stderr, "window %d: lazy minimum %.17g vs %.17g\n", w, m1, m2);
            mism++;
        }
        t0 += jump;
    }
    topowindow_free(win);
    /* orientation matters on this graph: pairs whose two rows disagree in the last bits */
    const int64_t A = shdtopo_num_attached(bat);
    double* lat = (double*)malloc(sizeof(double) * (size_t)(A * A));
    if (shdtopo_table_to_host(bat, lat, NULL, NULL) == 0)
        for (int64_t i = 0; i < A; i++)
            for (int64_t j = i + 1; j < A; j++)
                if (lat[i * A + j] != lat[j * A + i]) reversed++;
    printf("engine_window: %s, %ld packets in %d windows, %ld delivered, %ld mismatches, "
           "window %llu ns, %ld of %lld attached pairs orientation-dependent\n",
           serial ? "serial" : "multi-threaded", total, windows, delivered, mism,
           (unsigned long long)jump, reversed, (long long)(A * (A - 1) / 2));
    return mism ? 1 : 0;
}
