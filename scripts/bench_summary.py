"""One-screen summary of a bench.py JSON line: C2, C3 and the mixed legs
with their virtual-shard projections.  Usage: python scripts/bench_summary.py FILE"""
import json
import sys


def main():
    d = json.load(open(sys.argv[1]))
    print(f"C2 inflate {d['value']} GiB/s  kernel_ms {d['roofline']['kernel_ms']}  parity {d.get('parity_ok')}")
    df = d.get("deflate")
    if isinstance(df, dict):
        print(f"C3 deflate {df.get('deflate_value')}  roundtrip {df.get('roundtrip_value')}  ratio {df.get('ratio')}"
              f"  size/beast {df.get('size_vs_beast', df.get('beast_ratio'))}")
    m = d.get("mixed", {})
    for leg, v in m.items():
        if not isinstance(v, dict):
            continue
        print(f"{leg}: deflate {v.get('deflate_value')} inflate {v.get('inflate_value')} ratio {v.get('ratio_rank_local')}"
              f" ok {v.get('roundtrip_ok')}")
        for n, s in (v.get("virtual_shards") or {}).items():
            print(f"   N={n}: inflate {s.get('inflate_projected_speedup')}x (max shard "
                  f"{max(s.get('inflate_shard_ms', [0]))} ms)  deflate {s.get('deflate_projected_speedup')}x")


if __name__ == "__main__":
    main()
