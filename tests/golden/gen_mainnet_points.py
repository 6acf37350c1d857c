"""Generates tests/golden/mainnet_g2_points.json (+ _bad) from G2 points held as data in the
reference's own fixtures (run in the build container only; /root/reference is absent on
the GPU box).  Sources:
  packages/beacon-node/test/unit/sync/backfill/blocks.json   (mainnet block sigs + randao)
  packages/state-transition/test/unit/util/aggregator.test.ts
  packages/beacon-node/test/unit/chain/opPools/aggregatedAttestationPool.test.ts
  packages/state-transition/test/perf/util.ts
Points are classified by the oracle (decompress + psi subgroup check)."""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle.curves import g2_uncompress, in_g2_psi, BlstError  # noqa: E402

REF = "/root/reference/packages"


def main():
    pts = []
    for b in json.load(open(f"{REF}/beacon-node/test/unit/sync/backfill/blocks.json")):
        pts += [b["signature"][2:], b["message"]["body"]["randao_reveal"][2:]]
    for f in ["state-transition/test/unit/util/aggregator.test.ts",
              "beacon-node/test/unit/chain/opPools/aggregatedAttestationPool.test.ts",
              "state-transition/test/perf/util.ts"]:
        pts += re.findall(r"0x([0-9a-f]{192})\b", open(f"{REF}/{f}").read())
    good, bad = [], []
    for p in pts:
        try:
            ok = in_g2_psi(g2_uncompress(bytes.fromhex(p)))
            err = None if ok else "BLST_POINT_NOT_IN_GROUP"
        except BlstError as e:
            err = str(e)
        if err is None:
            if p not in good:
                good.append(p)
        else:
            bad.append({"sig": p, "error": err})
    json.dump(good, open(os.path.join(HERE, "mainnet_g2_points.json"), "w"), indent=1)
    json.dump(bad, open(os.path.join(HERE, "mainnet_g2_points_bad.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
