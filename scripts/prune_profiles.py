"""Fold the per-run bench logs of old session directories into one runs.jsonl each.

    python scripts/prune_profiles.py profiles/r02 profiles/r03

Every <session>/<run>.log that holds bench.py JSON lines and NOTHING else (blank lines
aside) becomes lines of <session>/runs.jsonl ({"run": <run>, **that JSON}) and is removed.
A log with any other output (rocprofv3 text, warnings, pytest, phase stamps), or with a
JSON line that does not parse, is left as it is and contributes nothing.  runs.jsonl is
rewritten keyed by run name, so folding a session twice changes nothing."""
import json
import os
import sys


def _bench_lines(path):
    """The parsed bench lines of a log made only of them, else None."""
    out = []
    for ln in open(path, errors="replace"):
        ln = ln.strip()
        if not ln:
            continue
        if not ln.startswith('{"metric"'):
            return None
        try:
            out.append(json.loads(ln))
        except ValueError:
            return None
    return out or None


def fold(session):
    jl = os.path.join(session, "runs.jsonl")
    runs = {}
    if os.path.exists(jl):
        for ln in open(jl):
            if ln.strip():
                r = json.loads(ln)
                runs.setdefault(r["run"], []).append(r)
    folded = []
    for f in sorted(os.listdir(session)):
        p = os.path.join(session, f)
        if not f.endswith(".log") or not os.path.isfile(p):
            continue
        lines = _bench_lines(p)
        if lines is None:
            continue
        runs[f[:-4]] = [dict(run=f[:-4], **d) for d in lines]
        folded.append(p)
    if folded:
        tmp = jl + ".tmp"
        with open(tmp, "w") as out:
            for name in sorted(runs):
                for r in runs[name]:
                    out.write(json.dumps(r) + "\n")
        os.replace(tmp, jl)
        for p in folded:  # removed only once runs.jsonl holds their lines
            os.remove(p)
    return len(folded)


if __name__ == "__main__":
    for root in sys.argv[1:]:
        for d in sorted(os.listdir(root)):
            p = os.path.join(root, d)
            if os.path.isdir(p):
                n = fold(p)
                if n:
                    print(p, n)
