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

Paths: "dense Ed25519" (cordahip_ed25519_verify_device over C2 corpora),
"dense ECDSA" (cordahip_ecdsa_verify_device over C3 corpora) and "stream" (C5
verifier-queue batches, 80% Ed25519 / 10% P-256 / 10% secp256k1, through
cordahip_stream_verify from pinned host memory); the ECDSA share counts the
dense ECDSA lanes and the stream batches' ECDSA sections. Logs given after
--rerun are re-runs of already counted batches on a later library: they are
not counted again, their GPU status digests must equal the counted ones.

usage: python tools/agree_combine.py LOG.jsonl... [--rerun LOG.jsonl...] > profiles/rNN_agreement_1e9.json
"""
import json
import subprocess
import sys


def main():
    recs = {}
    argv = sys.argv[1:]
    reruns = []
    if "--rerun" in argv:
        i = argv.index("--rerun")
        argv, reruns = argv[:i], argv[i + 1:]
    for path in argv:
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
    rerun_checks = []
    for path in reruns:
        with open(path) as f:
            for line in f:
                r = json.loads(line)
                key = (r["scheme"], r["batch"])
                if key not in recs:
                    raise SystemExit("re-run batch %s was never counted" % (key,))
                rerun_checks.append({"scheme": r["scheme"], "batch": r["batch"], "log": path,
                                     "oracle_mismatches": r["oracle_mismatches"],
                                     "construction_mismatches": r["construction_mismatches"],
                                     "gpu_digest_equals_counted": r["gpu_status_sha256"] == recs[key]["gpu_status_sha256"]})
    lanes = sum(t["lanes"] for t in tot.values())
    ec_lanes = tot.get("ecdsa", {}).get("lanes", 0) + sum(
        r.get("ecdsa_lanes", 0) for (sch, _), r in recs.items() if sch == "stream")
    paths = {"dense_ed25519": tot.get("ed25519", {}).get("lanes", 0), "dense_ecdsa": tot.get("ecdsa", {}).get("lanes", 0),
             "stream": tot.get("stream", {}).get("lanes", 0), "ecdsa_lanes_all_paths": ec_lanes,
             "ecdsa_share": ec_lanes / lanes if lanes else 0.0}
    checked = sum(t["oracle_checked"] for t in tot.values())
    mism = sum(t["oracle_mismatches"] + t["construction_mismatches"] for t in tot.values())
    try:
        head = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True).strip()
    except Exception:  # noqa: BLE001
        head = None
    mism += sum(c["oracle_mismatches"] + c["construction_mismatches"] + (not c["gpu_digest_equals_counted"])
                for c in rerun_checks)
    out = {"lanes": lanes, "oracle_checked": checked, "mismatches": mism, "all_lanes_oracle_checked": checked == lanes,
           "per_path": paths, "per_scheme": tot, "reruns": rerun_checks, "combined_at_commit": head,
           "note": "tools/agree_1e9.py --oracle-all in slices on one MI355X box per slice: every lane's status byte vs "
                   "the C oracle (and vs the corpus construction where it fixes the status); C2 corpora (Ed25519, 1% "
                   "corrupted/non-canonical/off-curve/small-order/S+kL) and C3 corpora (secp256k1/P-256 50/50, DER "
                   "malformations, r/s out of range, off-curve and compressed keys, high-S), one fresh seed per batch; "
                   "stream batches: a C2 corpus (80%) and a C3 corpus (20%) as one C5 queue through "
                   "cordahip_stream_verify",
           "batches": [dict(r) for _, r in sorted(recs.items())]}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
