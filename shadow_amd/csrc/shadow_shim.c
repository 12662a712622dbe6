/*
 * shadow_shim.c -- libshdtopo_shim.so: minimal restatements of the four Shadow functions that
 * libshdtopo.so imports (include/shd_topology_abi.h), for driving the library outside the
 * Shadow executable (tests, bench).  Inside Shadow the real definitions win.
 *
 *   address_toNetworkIP       src/topology/shd-address.c:114-117  (Address holds a network-order IP)
 *   random_new / nextDouble   src/utility/shd-random.c:13-37      (glibc rand_r stream)
 *   worker_updateMinTimeJump  src/engine/shd-worker.c:459 -> shd-master.c:113-124 (recorded)
 *   logging_log               src/support/shd-logging.c:127-135 (recorded; printed to stderr at
 *                             the SHDTOPO_LOG level: 1 critical + warning, 2 + message, 3 + info)
 * Shadow calls the last two from every worker thread: both are serialised by one mutex here.
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
void worker_updateMinTimeJump(double minPathLatency) {
    pthread_mutex_lock(&g_mu);
    g_last_min = minPathLatency;
    g_updates++;
    if (g_next_min_jump == 0 || minPathLatency < (double)g_next_min_jump)
        g_next_min_jump = ((uint64_t)minPathLatency) * 1000000ull;
    pthread_mutex_unlock(&g_mu);
}
double shim_last_min_latency(void) { return g_last_min; }
uint64_t shim_next_min_jump(void) { return g_next_min_jump; }
int shim_min_updates(void) { return g_updates; }
void shim_reset(void) {
    g_last_min = 0.0;
    g_next_min_jump = 0;
    g_updates = 0;
}

/* logging_log: the last kLogRing messages {GLib level, function, formatted text} are kept for tests
 * (tests/c/log_capture.c) */
#define kLogRing 64
typedef struct {
    int level;
    char func[64];
    char text[512];
} ShimLog;
static ShimLog g_log[kLogRing];
static int g_log_n = 0; /* messages logged since the last reset */
static int g_log_crit = 0; /* of which critical */
void logging_log(const char* log_domain, int log_level, const char* fileName,
                 const char* functionName, int lineNumber, const char* format, ...) {
    (void)log_domain;
    (void)fileName;
    (void)lineNumber;
    pthread_mutex_lock(&g_mu);
    ShimLog* e = &g_log[g_log_n % kLogRing];
    va_list ap;
    va_start(ap, format);
    vsnprintf(e->text, sizeof e->text, format, ap);
    va_end(ap);
    e->level = log_level;
    if (log_level == (1 << 3)) g_log_crit++;
    snprintf(e->func, sizeof e->func, "%s", functionName ? functionName : "n/a");
    g_log_n++;
    const char* env = getenv("SHDTOPO_LOG");
    const int want = env ? atoi(env) : 1;
    const int lvl = log_level <= (1 << 4) ? 1 : (log_level == (1 << 5) ? 2 : 3);
    if (lvl <= want) {
        const char* tag = log_level == (1 << 3) ? "critical"
                          : log_level == (1 << 4) ? "warning"
                          : log_level == (1 << 5) ? "message" : "info";
        fprintf(stderr, "[shadow] %s: [%s] %s\n", tag, e->func, e->text);
    }
    pthread_mutex_unlock(&g_mu);
}
int shim_log_count(void) { return g_log_n; }
int shim_log_criticals(void) { return g_log_crit; }
/* the i-th most recent message (0 = last): its text, level and function; -1 if not kept */
int shim_log_get(int i, int* level, char* func, int funcCap, char* text, int textCap) {
    if (i < 0 || i >= g_log_n || i >= kLogRing) return -1;
    const ShimLog* e = &g_log[(g_log_n - 1 - i) % kLogRing];
    if (level) *level = e->level;
    if (func && funcCap > 0) snprintf(func, (size_t)funcCap, "%s", e->func);
    if (text && textCap > 0) snprintf(text, (size_t)textCap, "%s", e->text);
    return 0;
}
void shim_log_reset(void) {
    pthread_mutex_lock(&g_mu);
    g_log_n = 0;
    g_log_crit = 0;
    pthread_mutex_unlock(&g_mu);
}
