// Host check of HostPrep::tree_order (topo_internal.h): on random parent forests (vertex 0 a root,
// other roots, deep chains, wide fans) the preorder must equal the order of the root-first parent
// paths compared lexicographically -- what the source grouping sorted by before round 6 -- and
// depth the number of parent hops to the root.  Prints "ok" and exits 0, or the first mismatch.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../shadow_amd/csrc/topo_internal.h"

using shdtopo::HostPrep;

static int check(uint32_t V, uint32_t seed, double p_root) {
    std::mt19937 rng(seed);
    HostPrep hp;
    hp.sptPar.assign(V, 0xFFFFFFFFu);
    // parents among earlier vertices of a random permutation: a forest with any id order
    std::vector<uint32_t> order(V);
    for (uint32_t i = 0; i < V; i++) order[i] = i;
    std::shuffle(order.begin() + 1, order.end(), rng);  // vertex 0 first: always a root
    std::uniform_real_distribution<double> u(0.0, 1.0);
    for (uint32_t i = 1; i < V; i++) {
        if (u(rng) < p_root) continue;
        const uint32_t lo = i > 40 && u(rng) < 0.5 ? i - 40 : 0;  // deep chains and wide fans
        hp.sptPar[order[i]] = order[lo + rng() % (i - lo)];
    }
    shdtopo::tree_order(hp);
    std::vector<std::vector<uint32_t>> path(V);
    for (uint32_t v = 0; v < V; v++) {
        for (uint32_t x = v; x != 0xFFFFFFFFu; x = hp.sptPar[x]) path[v].push_back(x);
        std::reverse(path[v].begin(), path[v].end());
        if (hp.depth[v] != path[v].size() - 1) {
            printf("depth mismatch at %u: %u vs %zu\n", v, hp.depth[v], path[v].size() - 1);
            return 1;
        }
    }
    std::vector<uint32_t> byPath(V), byPre(V);
    for (uint32_t i = 0; i < V; i++) byPath[i] = byPre[i] = i;
    std::stable_sort(byPath.begin(), byPath.end(), [&](uint32_t a, uint32_t b) {
        return std::lexicographical_compare(path[a].begin(), path[a].end(), path[b].begin(),
                                            path[b].end());
    });
    std::stable_sort(byPre.begin(), byPre.end(),
                     [&](uint32_t a, uint32_t b) { return hp.preorder[a] < hp.preorder[b]; });
    if (byPath != byPre) {
        printf("order mismatch (V %u seed %u)\n", V, seed);
        return 1;
    }
    return 0;
}

int main() {
    const uint32_t sizes[] = {1, 2, 3, 17, 200, 5000};
    for (uint32_t V : sizes)
        for (uint32_t seed = 1; seed <= 4; seed++)
            for (double pr : {0.0, 0.01, 0.3})
                if (check(V, seed, pr)) return 1;
    printf("ok\n");
    return 0;
}
