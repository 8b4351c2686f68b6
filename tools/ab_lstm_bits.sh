cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
TAM_LIB_PATH=$PWD/tiresias_amd/_C_base.so timeout -k 10 120 python -u tools/diag_lstm_bits.py base || exit 1
timeout -k 10 120 python -u tools/diag_lstm_bits.py new || exit 1
python - <<'PY'
import torch
a = torch.load("gpurun_out/lstm_bits_base.pt"); b = torch.load("gpurun_out/lstm_bits_new.pt")
for k in ("rev0", "rev1"):
    for n in ("hs", "cs", "act", "dG"):
        x, y = a[k][n].float(), b[k][n].float()
        print(k, n, "equal" if torch.equal(x, y) else f"DIFF max {float((x - y).abs().max()):.3e} at {int((x - y).abs().argmax())}")
print("gnmt loss", a["gnmt"]["loss"], b["gnmt"]["loss"], "grad equal", torch.equal(a["gnmt"]["grad"], b["gnmt"]["grad"]),
      float((a["gnmt"]["grad"] - b["gnmt"]["grad"]).norm() / a["gnmt"]["grad"].norm()))
for tag, d in (("base", a), ("new", b)):
    print(tag, "same-build rerun grad equal", torch.equal(d["gnmt"]["grad"], d["gnmt"]["grad_again"]))
ga, gb = a["gnmt"]["grad"], b["gnmt"]["grad"]
rows = []
for name, off, n in a["gnmt"]["params"]:
    x, y = ga[off:off + n], gb[off:off + n]
    rows.append((float((x - y).norm() / (x.norm() + 1e-30)), name))
rows.sort(reverse=True)
print("params differing:", sum(r[0] > 0 for r in rows), "of", len(rows))
for r in rows[:8]:
    print(f"  {r[0]:.3e} {r[1]}")
PY
rm -f gpurun_out/lstm_bits_*.pt
