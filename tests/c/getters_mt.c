/*
 * getters_mt.c -- the drop-in getters under Shadow's threading contract, through the C ABI.
 *
 * Shadow calls topology_getReliability / topology_getLatency / topology_isRoutable concurrently
 * from every worker thread (src/engine/shd-worker.c:179-203 start the workers, :352,360 call the
 * getters per packet; src/host/shd-host.c:1082 calls isRoutable); the reference serialises them
 * with its RW locks (src/topology/shd-topology.c:455-467,514-531).  Here T worker threads hammer
 * the getters of one lazy-mode topology (non-complete, >= 2,000 vertices) from before its first
 * table exists -- so the first getters race into the build -- while the main thread attaches a
 * second batch of hosts on NEW vertices mid-run (the table is rebuilt under the readers).
 *
 * Checked:
 *   * every answer (latency, reliability) equals the final table's T[s][d] or, the topology being
 *     undirected, T[d][s] bit for bit (first-rooted-wins orientation), and every
 *     isRoutable is 1;
 *   * at a quiescent barrier before the late attach: the lazy running minimum equals the minimum,
 *     over the rows materialised so far, of their row minima over the columns attached then, and
 *     each row's offered minimum equals that row minimum;
 *   * at the end: the lazy minimum equals the minimum of the offered row minima; each offered
 *     minimum is a value of its row and lies between the row's minimum over the final columns and
 *     over the first-batch columns; topology_getMinimumLatency equals the final table's minimum;
 *   * no critical log line, no crash.
 *
 * usage: getters_mt [integer_latency threads queries_per_thread]   exit 0 = pass, 1 = mismatch
 * Test infrastructure: links libshdtopo.so + libshdtopo_shim.so only (no oracle).
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shd_topology_abi.h"

Address* shim_address_new(uint32_t networkIP);
Random* random_new(unsigned int seed);
int shim_log_criticals(void);

enum { kRouters = 2600, kPoi = 400, kEdges = 26000, kPoiA = 300, kHostsPerPoiA = 2 };

typedef struct {
    Address* addr;
    uint32_t ip;
    int32_t vertex;
} Host;

static Topology* g_top;
static Host* g_hosts;
static int g_nA, g_nAll;           /* hosts of the first batch, of both batches */
static atomic_int g_lateDone;      /* the late batch is attached: queries may name it */
static pthread_barrier_t g_bar;
static int g_queries;

typedef struct {
    int id;
    int32_t* s;
    int32_t* d;
    double* lat;
    double* rel;
    int* routable;
    int n;
} Work;

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static void* worker(void* arg) {
    Work* w = (Work*)arg;
    uint64_t r = mix((uint64_t)w->id * 7919u + 1u);
    for (int k = 0; k < g_queries; k++) {
        if (k == g_queries / 2) { /* quiescent check by the main thread, then the late attach */
            pthread_barrier_wait(&g_bar);
            pthread_barrier_wait(&g_bar);
        }
        const int pool = atomic_load(&g_lateDone) ? g_nAll : g_nA;
        r = mix(r);
        const int s = (int)(r % (uint64_t)pool);
        int d = (int)((r >> 32) % (uint64_t)(pool - 1));
        if (d >= s) d++;
        /* shd-worker.c:352 then :360 (the latency only for a delivered packet: always here) */
        const double rel = topology_getReliability(g_top, g_hosts[s].addr, g_hosts[d].addr);
        const double lat = topology_getLatency(g_top, g_hosts[s].addr, g_hosts[d].addr);
        const int ok = topology_isRoutable(g_top, g_hosts[s].addr, g_hosts[d].addr);
        w->s[w->n] = s;
        w->d[w->n] = d;
        w->lat[w->n] = lat;
        w->rel[w->n] = rel;
        w->routable[w->n] = ok;
        w->n++;
    }
    return NULL;
}

static void poi_ip(int k, char* buf, size_t cap) { /* the generator's poi-k address */
    const unsigned a = (unsigned)k + 1u;
    snprintf(buf, cap, "10.%u.%u.%u", (a >> 16) & 255u, (a >> 8) & 255u, a & 255u);
}

static void attach_host(int h, int poi) {
    char hint[32];
    poi_ip(poi, hint, sizeof hint);
    g_hosts[h].ip = 11u | ((uint32_t)(h >> 8) << 16) | ((uint32_t)((h & 255) + 1) << 24);
    g_hosts[h].addr = shim_address_new(g_hosts[h].ip);
    Random* rnd = random_new((unsigned)(h + 1)); /* not drawn from: an exact ipHint match */
    topology_attach(g_top, g_hosts[h].addr, rnd, hint, NULL, NULL, NULL, NULL);
    g_hosts[h].vertex = shdtopo_vertex_of_ip(g_top, g_hosts[h].ip);
}

static int64_t col_of(const int32_t* cols, int64_t A, int32_t v) {
    int64_t lo = 0, hi = A;
    while (lo < hi) {
        const int64_t m = (lo + hi) / 2;
        if (cols[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo < A && cols[lo] == v ? lo : -1;
}

static int same(double a, double b) { return memcmp(&a, &b, sizeof a) == 0; }

int main(int argc, char** argv) {
    const int integer = argc > 1 ? atoi(argv[1]) : 0;
    const int nth = argc > 2 ? atoi(argv[2]) : 16;
    g_queries = argc > 3 ? atoi(argv[3]) : 20000;
    ShdSynthParams p = {integer ? 777ull : 778ull, kRouters, kPoi, kEdges, integer, 1.0 / 1.1, 0};
    g_top = shdtopo_new_synthetic(&p);
    if (!g_top) return 2;
    shdtopo_set_option(g_top, "lazy", 1);
    g_nA = kPoiA * kHostsPerPoiA;
    g_nAll = g_nA + (kPoi - kPoiA);
    g_hosts = (Host*)calloc((size_t)g_nAll, sizeof(Host));
    for (int h = 0; h < g_nA; h++) attach_host(h, h % kPoiA);
    long bad = 0;
    pthread_barrier_init(&g_bar, NULL, (unsigned)nth + 1);
    Work* w = (Work*)calloc((size_t)nth, sizeof(Work));
    pthread_t* th = (pthread_t*)calloc((size_t)nth, sizeof(pthread_t));
    for (int t = 0; t < nth; t++) {
        w[t].id = t;
        w[t].s = (int32_t*)malloc(sizeof(int32_t) * (size_t)g_queries);
        w[t].d = (int32_t*)malloc(sizeof(int32_t) * (size_t)g_queries);
        w[t].lat = (double*)malloc(sizeof(double) * (size_t)g_queries);
        w[t].rel = (double*)malloc(sizeof(double) * (size_t)g_queries);
        w[t].routable = (int*)malloc(sizeof(int) * (size_t)g_queries);
        pthread_create(&th[t], NULL, worker, &w[t]); /* no table yet: they race into the build */
    }

    /* ---- quiescent point: every worker waits at the second barrier ---- */
    pthread_barrier_wait(&g_bar);
    {
        const int64_t A1 = shdtopo_num_attached(g_top);
        int32_t* c1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)A1);
        double* T1 = (double*)malloc(sizeof(double) * (size_t)(A1 * A1));
        shdtopo_attached_vertices(g_top, c1, A1);
        if (A1 != kPoiA || shdtopo_table_to_host(g_top, T1, NULL, NULL) != 0) {
            fprintf(stderr, "first-batch table: A = %lld (expected %d)\n", (long long)A1, kPoiA);
            return 1;
        }
        const int64_t n1 = shdtopo_lazy_rows(g_top, NULL, NULL, NULL, 0);
        int32_t* v1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n1 + 1));
        double* m1 = (double*)malloc(sizeof(double) * (size_t)(n1 + 1));
        shdtopo_lazy_rows(g_top, v1, NULL, m1, n1);
        double expect = INFINITY;
        for (int64_t i = 0; i < n1; i++) {
            const int64_t c = col_of(c1, A1, v1[i]);
            double m = INFINITY;
            for (int64_t j = 0; c >= 0 && j < A1; j++)
                if (T1[c * A1 + j] < m) m = T1[c * A1 + j];
            if (c < 0 || !same(m, m1[i])) {
                if (bad < 5)
                    fprintf(stderr, "first batch: row %d offered %.17g, row minimum %.17g\n", v1[i],
                            m1[i], m);
                bad++;
            }
            if (m < expect) expect = m;
        }
        const double lm = shdtopo_get_lazy_minimum_latency(g_top);
        if (!same(lm, expect)) {
            fprintf(stderr, "first batch: lazy minimum %.17g, materialised rows' minimum %.17g\n",
                    lm, expect);
            bad++;
        }
        printf("getters_mt: quiescent point: %lld of %d rows materialised, lazy minimum %.17g\n",
               (long long)n1, kPoiA, lm);
        free(c1);
        free(T1);
        free(v1);
        free(m1);
    }
    pthread_barrier_wait(&g_bar); /* the workers resume */

    /* late attach: kPoi - kPoiA hosts on new vertices while the workers query */
    for (int h = g_nA; h < g_nAll; h++) attach_host(h, kPoiA + (h - g_nA));
    atomic_store(&g_lateDone, 1);
    for (int t = 0; t < nth; t++) pthread_join(th[t], NULL);

    /* ---- final state ---- */
    const int64_t A = shdtopo_num_attached(g_top);
    int32_t* cols = (int32_t*)malloc(sizeof(int32_t) * (size_t)A);
    shdtopo_attached_vertices(g_top, cols, A);
    double* T = (double*)malloc(sizeof(double) * (size_t)(A * A));
    double* R = (double*)malloc(sizeof(double) * (size_t)(A * A));
    if (A != kPoi || shdtopo_table_to_host(g_top, T, R, NULL) != 0) {
        fprintf(stderr, "final table: A = %lld (expected %d)\n", (long long)A, kPoi);
        return 1;
    }
    /* answers */
    long total = 0, reversed = 0;
    for (int t = 0; t < nth; t++)
        for (int k = 0; k < w[t].n; k++) {
            total++;
            const int64_t cs = col_of(cols, A, g_hosts[w[t].s[k]].vertex);
            const int64_t cd = col_of(cols, A, g_hosts[w[t].d[k]].vertex);
            const int64_t f = cs * A + cd, b = cd * A + cs;
            const int fwd = same(w[t].lat[k], T[f]) && same(w[t].rel[k], R[f]);
            const int rev = same(w[t].lat[k], T[b]) && same(w[t].rel[k], R[b]);
            if (!fwd && rev) reversed++;
            if (cs < 0 || cd < 0 || (!fwd && !rev) || w[t].routable[k] != 1) {
                if (bad < 5)
                    fprintf(stderr, "thread %d query %d (%d -> %d): %.17g / %.17g, table %.17g / "
                            "%.17g or %.17g / %.17g, routable %d\n", t, k, w[t].s[k], w[t].d[k],
                            w[t].lat[k], w[t].rel[k], T[f], R[f], T[b], R[b], w[t].routable[k]);
                bad++;
            }
        }
    /* lazy minimum vs the materialised rows */
    const int64_t nm = shdtopo_lazy_rows(g_top, NULL, NULL, NULL, 0);
    int32_t* mv = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nm + 1));
    uint64_t* me = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(nm + 1));
    double* mm = (double*)malloc(sizeof(double) * (size_t)(nm + 1));
    shdtopo_lazy_rows(g_top, mv, me, mm, nm);
    double expect = INFINITY;
    for (int64_t i = 0; i < nm; i++) {
        const int64_t c = col_of(cols, A, mv[i]);
        if (c < 0) { bad++; continue; }
        double mAll = INFINITY, mFirst = INFINITY;
        int member = 0;
        for (int64_t j = 0; j < A; j++) {
            const double x = T[c * A + j];
            if (x < mAll) mAll = x;
            if (cols[j] < kRouters + kPoiA && x < mFirst) mFirst = x; /* a first-batch column */
            member |= same(x, mm[i]);
        }
        if (!member || mm[i] < mAll || mm[i] > mFirst) {
            if (bad < 5)
                fprintf(stderr, "row %d: offered minimum %.17g, row minima %.17g (final) %.17g "
                        "(first batch)\n", mv[i], mm[i], mAll, mFirst);
            bad++;
        }
        if (mm[i] < expect) expect = mm[i];
    }
    const double lazyMin = shdtopo_get_lazy_minimum_latency(g_top);
    if (!same(lazyMin, expect)) {
        fprintf(stderr, "lazy minimum %.17g, materialised rows' minimum %.17g\n", lazyMin, expect);
        bad++;
    }
    double gmin = INFINITY;
    for (int64_t i = 0; i < A * A; i++)
        if (T[i] >= 0 && T[i] < gmin) gmin = T[i];
    const double eager = topology_getMinimumLatency(g_top);
    if (!same(eager, gmin)) {
        fprintf(stderr, "getMinimumLatency %.17g, table minimum %.17g\n", eager, gmin);
        bad++;
    }
    const int crit = shim_log_criticals();
    if (crit) {
        fprintf(stderr, "%d critical log lines\n", crit);
        bad++;
    }
    ShdStats st;
    shdtopo_get_stats(g_top, &st);
    printf("getters_mt: %s latencies, %d threads, %ld queries x 3 getters, %ld answered from the "
           "reverse row, %lld rows materialised, %lld rows copied to the host (%.1f ms), lazy min "
           "%.17g, %ld mismatches\n", integer ? "integer" : "real", nth, total, reversed,
           (long long)nm, (long long)st.rows_to_host, st.rows_to_host_ms, lazyMin, bad);
    topology_free(g_top);
    return bad ? 1 : 0;
}
