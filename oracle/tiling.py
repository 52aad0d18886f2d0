"""Oracle (test infrastructure): the min-cost tiling choice of
spartan/expr/tiling.cc restated in Python, to check libspx's
spx_mincost_tiling.

Follows find_mincost_tiling (tiling.cc:31-92) step by step: head-inserted
adjacency lists (an edge list is walked newest first, tiling.cc:19-22), the
split-pair lookup further down the list (:46), the "only one half reachable"
case (:48-55), the choose-one case with copies of the visited set and the
deferred tie (:56-79), and the ordinary consumer (:81-88); mincost_tiling
(:94-132) returns the visited nodes below t.

Parity is UNPINNED beyond this restatement: the reference module cannot be
built here (it is a Python-2 C extension: PyInt_AsLong tiling.cc:101,
Py_InitModule :141) and the reference ships no test or fixture for it.
"""

INF = 1000000000


def mincost_tiling(t, edges, split_pairs):
  """t: sink id; edges: [(u, v, cost)] in insertion order; split_pairs:
  [(a, b)].  Returns (sorted chosen node ids < t, total cost)."""
  head = {}
  nxt = []
  dst = []
  cst = []
  for (u, v, c) in edges:
    nxt.append(head.get(u, -1))
    dst.append(v)
    cst.append(c)
    head[u] = len(dst) - 1
  split = {}
  for a, b in split_pairs:
    split[a] = b
    split[b] = a
  dis = {}

  def find(s, vis):
    total = 0
    child = []
    i = head.get(s, -1)
    while i != -1:
      child.append(i)
      i = nxt[i]
    size = len(child)
    while child:
      i = child.pop(0)
      size -= 1
      v = dst[i]
      if v in split:
        sp = split[v]
        j = nxt[i]
        while j != -1 and dst[j] != sp:
          j = nxt[j]
        if j < 0:
          if vis[v] or vis[sp]:
            total += cst[i] if vis[v] else INF
          else:
            dis[v] = find(v, vis)
            total += dis[v] + cst[i]
            vis[v] = True
        else:
          if j in child:  # std::list::remove: a no-op when absent
            child.remove(j)
          size -= 1
          if vis[v] or vis[sp]:
            total += cst[i] if vis[v] else cst[j]
          else:
            vis1 = list(vis)
            vis2 = list(vis)
            dis[v] = find(v, vis1)
            dis[sp] = find(sp, vis2)
            cmp = dis[v] + cst[i] - dis[sp] - cst[j]
            if cmp == 0 and size > 0:
              child.append(i)
              child.append(j)
            elif cmp < 0:
              total += dis[v] + cst[i]
              vis[:] = vis1
              vis[v] = True
            else:
              total += dis[sp] + cst[j]
              vis[:] = vis2
              vis[sp] = True
      else:
        if vis[v]:
          total += cst[i]
        else:
          dis[v] = find(v, vis)
          total += dis[v] + cst[i]
          vis[v] = True
    return total

  vis = [False] * (t + 1)
  cost = find(0, vis)
  return [u for u in range(t) if vis[u]], cost
