/*
 * getter_bench.c -- libgetter_bench.so: the per-packet getter path timed as Shadow's workers drive
 * it (bench.py's "getters" block).  n queries, each the pair unchanged Shadow issues per packet
 * (src/engine/shd-worker.c:352 topology_getReliability, :360 topology_getLatency), are split over
 * nthreads pthreads that call the product's C ABI concurrently; answers are written out for the
 * caller's checks.  Address objects are made before the timed loop (Shadow's hosts own theirs).
 * Bench infrastructure: links libshdtopo.so + libshdtopo_shim.so only (no oracle).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include "../../include/shd_topology_abi.h"

Address* shim_address_new(uint32_t networkIP);
void shim_address_free(Address* a);

typedef struct {
    Topology* top;
    Address** src;
    Address** dst;
    double *lat, *rel;
    int64_t lo, hi, failed;
    struct timespec t0, t1;
    pthread_barrier_t* bar;
} Arg;

static void* run(void* a_) {
    Arg* a = (Arg*)a_;
    pthread_barrier_wait(a->bar);
    clock_gettime(CLOCK_MONOTONIC, &a->t0);
    for (int64_t i = a->lo; i < a->hi; i++) {
        a->rel[i] = topology_getReliability(a->top, a->src[i], a->dst[i]);
        a->lat[i] = topology_getLatency(a->top, a->src[i], a->dst[i]);
        a->failed += a->lat[i] < 0;
    }
    clock_gettime(CLOCK_MONOTONIC, &a->t1);
    return NULL;
}

/* Returns the wall nanoseconds of the query loop (first thread start to last thread end), or -1
 * when a query failed (an unattached address: the getters returned -1). */
int64_t getbench_run(Topology* top, int64_t n, const uint32_t* srcIP, const uint32_t* dstIP,
                     int nthreads, double* lat, double* rel) {
    if (!top || n <= 0 || nthreads < 1) return -1;
    Address** src = (Address**)malloc(sizeof(Address*) * (size_t)n);
    Address** dst = (Address**)malloc(sizeof(Address*) * (size_t)n);
    for (int64_t i = 0; i < n; i++) {
        src[i] = shim_address_new(srcIP[i]);
        dst[i] = shim_address_new(dstIP[i]);
    }
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    Arg* a = (Arg*)calloc((size_t)nthreads, sizeof(Arg));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (int t = 0; t < nthreads; t++) {
        a[t].top = top;
        a[t].src = src;
        a[t].dst = dst;
        a[t].lat = lat;
        a[t].rel = rel;
        a[t].lo = n * t / nthreads;
        a[t].hi = n * (t + 1) / nthreads;
        a[t].bar = &bar;
        pthread_create(&th[t], NULL, run, &a[t]);
    }
    int64_t t0 = INT64_MAX, t1 = 0, failed = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        const int64_t s = (int64_t)a[t].t0.tv_sec * 1000000000 + a[t].t0.tv_nsec;
        const int64_t e = (int64_t)a[t].t1.tv_sec * 1000000000 + a[t].t1.tv_nsec;
        if (s < t0) t0 = s;
        if (e > t1) t1 = e;
        failed += a[t].failed;
    }
    pthread_barrier_destroy(&bar);
    for (int64_t i = 0; i < n; i++) {
        shim_address_free(src[i]);
        shim_address_free(dst[i]);
    }
    free(src);
    free(dst);
    free(th);
    free(a);
    return failed ? -1 : t1 - t0;
}
