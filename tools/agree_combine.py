"""Combine the per-batch logs of the fully oracle-checked agreement sweep
(tools/agree_1e9.py --oracle-all --log, run in slices on the GPU box: a gpurun
call is capped at 20 minutes and the C oracle checks ~0.3 M Ed25519 / ~0.07 M
ECDSA lanes per second on the box's 16 host threads) into
profiles/r03_agreement_1e9.json.

Every batch is a fresh seeded corpus (seed = base + batch index, so slices
never overlap); every lane's GPU status byte was compared with the C oracle's
(oracle/c: i2p 0.2.0 / BouncyCastle 1.57 restatements) and with the corpus
construction where it fixes the status. The per-batch SHA-256 digests of both
status vectors are kept: equal digests = identical status bytes.

usage: python tools/agree_combine.py profiles/r03_agreement/*.jsonl > profiles/r03_agreement_1e9.json
"""
import json
import subprocess
import sys


def main():
    recs = {}
    for path in sys.argv[1:]:
        with open(path) as f:
            for line in f:
                r = json.loads(line)
                key = (r["scheme"], r["batch"])
                if key in recs:
                    raise SystemExit("batch %s appears twice" % (key,))
                r["log"] = path
                recs[key] = r
    tot = {}
    for (scheme, _), r in sorted(recs.items()):
        t = tot.setdefault(scheme, dict(batches=0, lanes=0, oracle_checked=0, construction_mismatches=0,
                                        oracle_mismatches=0, rejected=0, digest_mismatches=0))
        t["batches"] += 1
        t["lanes"] += r["lanes"]
        t["oracle_checked"] += r["oracle_checked"]
        t["construction_mismatches"] += r["construction_mismatches"]
        t["oracle_mismatches"] += r["oracle_mismatches"]
        t["rejected"] += r["rejected"]
        t["digest_mismatches"] += int(r["gpu_status_sha256"] != r["oracle_status_sha256"])
    lanes = sum(t["lanes"] for t in tot.values())
    checked = sum(t["oracle_checked"] for t in tot.values())
    mism = sum(t["oracle_mismatches"] + t["construction_mismatches"] for t in tot.values())
    try:
        head = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True).strip()
    except Exception:  # noqa: BLE001
        head = None
    out = {"lanes": lanes, "oracle_checked": checked, "mismatches": mism, "all_lanes_oracle_checked": checked == lanes,
           "per_scheme": tot, "combined_at_commit": head,
           "note": "tools/agree_1e9.py --oracle-all in slices on one MI355X box per slice: every lane's status byte vs "
                   "the C oracle (and vs the corpus construction where it fixes the status); C2 corpora (Ed25519, 1% "
                   "corrupted/non-canonical/off-curve/small-order/S+kL) and C3 corpora (secp256k1/P-256 50/50, DER "
                   "malformations, r/s out of range, off-curve and compressed keys, high-S), one fresh seed per batch",
           "batches": [dict(r) for _, r in sorted(recs.items())]}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
