"""Per-kernel and per-copy-direction summary (calls, average and total ns) of a rocprofv3 rocpd
database (rocprofv3 ... -d DIR -o run writes DIR/run_results.db), optionally over the last
dispatches only (SKIP=n skips the first n of each kernel)."""
import collections
import sqlite3
import sys


def tables(cur):
    names = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    pick = lambda p: [t for t in names if t.startswith(p)][0]
    return (pick("rocpd_kernel_dispatch"), pick("rocpd_info_kernel_symbol"),
            pick("rocpd_memory_copy"))


def main(path, skip=0):
    cur = sqlite3.connect(path).cursor()
    kd, ks, mc = tables(cur)
    rows = cur.execute(f"select s.display_name, d.start, d.end from {kd} d join {ks} s "
                       f"on d.kernel_id = s.id order by d.start").fetchall()
    per = collections.defaultdict(list)
    for name, a, b in rows:
        per[name].append(b - a)
    print(f"{'kernel':70s} {'calls':>6s} {'avg ns':>10s} {'total ms':>9s}")
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        v = v[skip:] or v
        print(f"{name[:70]:70s} {len(v):6d} {sum(v) / len(v):10.0f} {sum(v) / 1e6:9.3f}")
    cp = collections.defaultdict(list)
    for a, b, size, src, dst in cur.execute(f"select start, end, size, src_agent_id, "
                                            f"dst_agent_id from {mc}"):
        cp[(src, dst)].append((b - a, size))
    for k, v in cp.items():
        t = sum(x for x, _ in v)
        s = sum(y for _, y in v)
        print(f"copy agent {k[0]}->{k[1]}: {len(v)} copies, {s / 1e6:.1f} MB, {t / 1e6:.3f} ms, "
              f"{s / max(t, 1):.1f} GB/s")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
