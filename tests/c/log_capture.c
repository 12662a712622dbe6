/*
 * log_capture.c -- the library's log lines reach Shadow's logger (src/support/shd-logging.h:24-67:
 * critical() / warning() / message() -> logging_log), and topology_free reports the reference's
 * shortest-path total like _topology_clearCache (src/topology/shd-topology.c:445-446):
 *     "path cache cleared, spent %f seconds computing %u shortest paths"
 * Linked like a Shadow build: libshdtopo.so + libshdtopo_shim.so, whose logging_log records every
 * message (level, function, text).
 *
 * usage: log_capture GRAPHML [HOSTS]
 *   HOSTS = 0 (default, no GPU): load, query an unattached address (a critical line), free.
 *   HOSTS > 0 (GPU): also attach HOSTS hosts (no hints: the reference's random choice), query every
 *   pair (the table is built), free.  Prints the attached vertex count and the captured lines;
 *   exit 0 when the clearCache line carries the expected count, 1 otherwise.
 * Test infrastructure: no oracle.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shd_topology_abi.h"

Address* shim_address_new(uint32_t networkIP);
Random* random_new(unsigned int seed);
int shim_log_count(void);
int shim_log_get(int i, int* level, char* func, int funcCap, char* text, int textCap);

static int find(const char* needle, int* level, char* func, char* text) {
    for (int i = 0; i < shim_log_count() && i < 64; i++) {
        if (shim_log_get(i, level, func, 64, text, 512) == 0 && strstr(text, needle)) return 1;
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int hosts = argc > 2 ? atoi(argv[2]) : 0;
    Topology* top = topology_new(argv[1]);
    if (!top) {
        printf("topology_new failed\n");
        return 1;
    }
    int level = 0;
    char func[64], text[512];
    /* an unattached address: the reference logs critical() and returns -1 (shd-topology.c:882-892) */
    Address* nobody = shim_address_new(0x0100000Au);
    const double l0 = topology_getLatency(top, nobody, nobody);
    const int crit = find("not connected to topology", &level, func, text);
    printf("unattached latency %.1f, critical line %s (level %d, function %s)\n", l0,
           crit ? "captured" : "MISSING", crit ? level : 0, crit ? func : "-");
    int ok = l0 == -1.0 && crit && level == (1 << 3);
    int32_t nattached = 0;
    if (hosts > 0) {
        Random* rng = random_new(12345u);
        Address** a = (Address**)calloc((size_t)hosts, sizeof(Address*));
        for (int h = 0; h < hosts; h++) {
            a[h] = shim_address_new(0x0B000001u + (uint32_t)h);
            topology_attach(top, a[h], rng, NULL, NULL, NULL, NULL, NULL);
        }
        for (int s = 0; s < hosts; s++)
            for (int d = 0; d < hosts; d++) ok = ok && topology_getLatency(top, a[s], a[d]) > 0;
        nattached = (int32_t)shdtopo_num_attached(top);
    }
    topology_free(top);
    char want[96];
    snprintf(want, sizeof want, "computing %d shortest paths", (int)nattached);
    const int cc = find("path cache cleared", &level, func, text);
    printf("attached vertices %d\nclearCache line: %s (level %d, function %s)\n", (int)nattached,
           cc ? text : "MISSING", cc ? level : 0, cc ? func : "-");
    ok = ok && cc && level == (1 << 5) && strstr(text, want) != NULL;
    printf("%s\n", ok ? "log capture ok" : "log capture FAILED");
    return ok ? 0 : 1;
}
