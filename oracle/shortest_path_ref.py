"""CPU restatement of the ShortestPath heuristic's first hops — TEST INFRASTRUCTURE ONLY.

The reference takes shortest_paths[now][target][1] from
nx.shortest_path(G, weight="weight") (src/env/network.py:279, src/policy.py:119-137).
networkx 3.4.2 (the version in this image; pyproject pins networkx>=3.1) computes it
per source with _dijkstra_multisource: a heap of (distance, push counter, node), a
node's path replaced only on a strictly shorter tentative distance, neighbours relaxed
in G's adjacency order (the order edges were added = creation order,
src/env/network.py:179-186). Restated here with heapq; pinned against
tests/golden/shortest.npz (first-hop tables produced by the reference + networkx).
"""
import heapq

import numpy as np


def first_hop_table(n, edges):
    """edges: [(a, b, length)] in creation order -> int32 [n, n] first hops (t on the diagonal)."""
    adj = [[] for _ in range(n)]
    for a, b, ln in edges:
        adj[int(a)].append((int(b), int(ln)))
        adj[int(b)].append((int(a), int(ln)))
    first = np.zeros((n, n), np.int32)
    for src in range(n):
        dist, seen, hop = {}, {src: 0}, {src: src}
        c = 0
        fringe = [(0, c, src)]
        while fringe:
            d, _, v = heapq.heappop(fringe)
            if v in dist:
                continue
            dist[v] = d
            for u, ln in adj[v]:
                vu = d + ln
                if u in dist:
                    continue
                if u not in seen or vu < seen[u]:
                    seen[u] = vu
                    c += 1
                    heapq.heappush(fringe, (vu, c, u))
                    hop[u] = u if v == src else hop[v]
        for t in range(n):
            first[src, t] = hop[t]
    return first


def shortest_path_actions(now, target, nbr, first):
    """src/policy.py:119-137 for one env: now/target [A], nbr [N, 3] ascending ids."""
    act = np.zeros(len(now), np.int32)
    for i, (v, t) in enumerate(zip(now, target)):
        if v == t:
            continue
        nx_ = first[v, t]
        for k in range(nbr.shape[1]):
            if nbr[v, k] == nx_:
                act[i] = k + 1
                break
    return act
