#!/usr/bin/env python3
"""Self-time summary of a node --cpu-prof profile (V8 .cpuprofile JSON): top functions."""
import collections
import json
import sys

d = json.load(open(sys.argv[1]))
nodes = {n["id"]: n for n in d["nodes"]}
self_t = collections.Counter()
for s, t in zip(d["samples"], d["timeDeltas"]):
    cf = nodes[s]["callFrame"]
    self_t[(cf["functionName"] or "(anon)") + " " + cf["url"].split("/")[-1] + ":" + str(cf["lineNumber"])] += t
tot = sum(self_t.values())
for k, v in self_t.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 25):
    print(f"{v / tot * 100:5.1f}% {k}")
