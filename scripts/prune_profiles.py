"""Fold the per-run bench logs of old session directories into one runs.jsonl each.

    python scripts/prune_profiles.py profiles/r02 profiles/r03

Every <session>/<run>.log whose content holds a bench.py JSON line becomes one line of
<session>/runs.jsonl ({"run": <run>, **that JSON}); the log itself is removed.  Logs
without a bench line (pytest, smoke, phase stamps, traces) and every other file stay."""
import json
import os
import sys


def fold(session):
    runs = []
    for f in sorted(os.listdir(session)):
        p = os.path.join(session, f)
        if not f.endswith(".log") or not os.path.isfile(p) or f.startswith(("pytest", "smoke", "phases", "session")):
            continue
        lines = [l for l in open(p, errors="replace") if l.startswith('{"metric"')]
        if not lines:
            continue
        for l in lines:
            try:
                runs.append(dict(run=f[:-4], **json.loads(l)))
            except ValueError:
                break
        else:
            os.remove(p)
    if runs:
        with open(os.path.join(session, "runs.jsonl"), "a") as out:
            for r in runs:
                out.write(json.dumps(r) + "\n")
    return len(runs)


if __name__ == "__main__":
    for root in sys.argv[1:]:
        for d in sorted(os.listdir(root)):
            p = os.path.join(root, d)
            if os.path.isdir(p):
                n = fold(p)
                if n:
                    print(p, n)
