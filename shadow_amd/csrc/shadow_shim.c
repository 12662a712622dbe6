/*
 * shadow_shim.c -- libshdtopo_shim.so: minimal restatements of the four Shadow functions that
 * libshdtopo.so imports (include/shd_topology_abi.h), for driving the library outside the
 * Shadow executable (tests, bench).  Inside Shadow the real definitions win.
 *
 *   address_toNetworkIP       src/topology/shd-address.c:114-117  (Address holds a network-order IP)
 *   random_new / nextDouble   src/utility/shd-random.c:13-37      (glibc rand_r stream)
 *   worker_updateMinTimeJump  src/engine/shd-worker.c:459 -> shd-master.c:113-124 (recorded)
 */
#include <stdint.h>
#include <stdlib.h>

struct _Address {
    uint32_t ip; /* network order */
};
typedef struct _Address Address;

struct _Random {
    unsigned int seedState;
    unsigned int initialSeed;
};
typedef struct _Random Random;

Address* shim_address_new(uint32_t networkIP) {
    Address* a = (Address*)calloc(1, sizeof(Address));
    a->ip = networkIP;
    return a;
}
void shim_address_free(Address* a) { free(a); }
uint32_t address_toNetworkIP(Address* address) { return address->ip; }

Random* random_new(unsigned int seed) {
    Random* r = (Random*)calloc(1, sizeof(Random));
    r->initialSeed = seed;
    r->seedState = seed;
    return r;
}
void random_free(Random* r) { free(r); }
int random_nextInt(Random* r) { return rand_r(&r->seedState); }
double random_nextDouble(Random* r) {
    return (double)(((double)rand_r(&r->seedState)) / ((double)RAND_MAX));
}
unsigned int shim_random_state(Random* r) { return r->seedState; }

/* master_updateMinTimeJump keeps (u64)minLat * 1e6 ns when smaller (shd-master.c:113-124) */
static double g_last_min = 0.0;
static uint64_t g_next_min_jump = 0;
static int g_updates = 0;
void worker_updateMinTimeJump(double minPathLatency) {
    g_last_min = minPathLatency;
    g_updates++;
    if (g_next_min_jump == 0 || minPathLatency < (double)g_next_min_jump)
        g_next_min_jump = ((uint64_t)minPathLatency) * 1000000ull;
}
double shim_last_min_latency(void) { return g_last_min; }
uint64_t shim_next_min_jump(void) { return g_next_min_jump; }
int shim_min_updates(void) { return g_updates; }
void shim_reset(void) {
    g_last_min = 0.0;
    g_next_min_jump = 0;
    g_updates = 0;
}
