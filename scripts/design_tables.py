"""Regenerate the two number tables of the design document (drop-in per-call costs, the bench
line's legs) from profiles/r03/bench_default.json.  usage: python scripts/design_tables.py"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = json.load(open(os.path.join(ROOT, "profiles", "r03", "bench_default.json")))
L = d["legs"]
dp = L["dropin_per_call_us"]
un = dp["uncombined_8_threads"]


def drow(sym, key, size, label, cpu_key, note=""):
    r, u = dp[size], un[size]
    bold = "**" if label == "16 KiB" else ""
    return (f"| `{sym}` {label} | {r[key + '_gpu_us']:.0f} | {bold}{r[key + '_gpu_us_8_threads']:.1f}{bold}{note} | "
            f"{u[key + '_gpu_us_8_threads']:.1f} | {r.get(cpu_key, '—')} |")


rows = []
for sym, key, cpuk in (("crc32c", "crc32c", "crc32c_cpu_us"),
                       ("rd_kafka_lz4_compress", "lz4_compress", "lz4_compress_cpu_us"),
                       ("rd_kafka_lz4_decompress", "lz4_decompress", "lz4_decompress_cpu_us")):
    for size, label in (("16384B", "16 KiB"), ("65536B", "64 KiB"), ("1048576B", "1 MiB")):
        note = " (own streams by the size rule)" if (label == "1 MiB" and key != "lz4_compress") else ""
        rows.append(drow(sym, key, size, label, cpuk, note))
dtable = ("| symbol, size | 1 thread | 8 threads, combined | 8 threads, own streams (`RDK_HIP_COMBINE=0`) | "
          "reference code, 1 core |\n|---|---|---|---|---|\n" + "\n".join(rows) + "\n")


def g(k):
    return L[k]


def ta(v):
    r = v["roofline"]
    return round(r["traffic"] / r["alg_bytes_per_launch"], 2) if r.get("traffic") else None


def iss(v):
    return (v.get("roofline_issue") or {}).get("frac")


def trio(fmt, keys, f):
    return " / ".join(fmt.format(f(g(k))) for k in keys)


ff = ["writer_finalize_fast_16KiB_json", "writer_finalize_fast_64KiB_json", "writer_finalize_fast_256KiB_json"]
fe = ["writer_finalize_16KiB_json", "writer_finalize_64KiB_json", "writer_finalize_256KiB_json"]
cc = ["consumer_crc_verify_lz4f_decompress_16KiB", "consumer_crc_verify_lz4f_decompress_64KiB",
      "consumer_crc_verify_lz4f_decompress_256KiB"]
gb = lambda v: v["GB_per_s"]  # noqa: E731
km = lambda v: v["roofline"]["kernel_ms"]  # noqa: E731
fr = lambda v: v["roofline"]["frac"]  # noqa: E731
cpu = lambda k: (g(k).get("cpu_baseline") or {}).get("value")  # noqa: E731


def line(name, k, c="—"):
    v = g(k)
    r = v["roofline"]
    i = iss(v) if iss(v) is not None else (r.get("issue") or {}).get("frac_of_issue_ceiling")
    return f"  | {name} | {v['GB_per_s']:.4g} | {r['kernel_ms']:.3g} ms | {r['frac']:.4f} | {ta(v)} | {i} | {c} |"


head_ta = round(d["roofline"]["traffic"] / d["roofline"]["alg_bytes_per_launch"], 1)
pt = g("perf_tool_1M_x_100B_messages")
pp = g("producer_pipeline_1MiB_json_pcie")["GB_per_s_by_host_threads"]
c = g("crc32c_only_16KiB_batches")
cr = c["roofline"]
rows = [
    "  | line | GB/s | kernel time | HBM frac | traffic / alg | issue | CPU reference (16 thr) |",
    "  |---|---|---|---|---|---|---|",
    f"  | **headline: writer finalize, throughput compressor** (512 × 1 MiB, ratio {d['compression_ratio']} vs 2.819) | "
    f"**{d['value']:.1f}** | {d['roofline']['kernel_ms']:.2f} ms | {d['roofline']['frac']:.4f} | {head_ta} | "
    f"{d['roofline_issue']['frac']} | {d['cpu_baseline']['value']:.1f} |",
    line("writer finalize, byte-identical (round 2's headline)", "writer_finalize_1MiB_json",
         f"{cpu('writer_finalize_1MiB_json'):.1f}"),
    f"  | writer finalize fast, 32768 × 16 KiB / 8192 × 64 KiB / 2048 × 256 KiB | {trio('{:.1f}', ff, gb)} | "
    f"{trio('{:.2f}', ff, km)} ms | {trio('{:.3f}', ff, fr)} | {trio('{}', ff, ta)} | {trio('{}', ff, iss)} | — |",
    f"  | writer finalize exact, 16 KiB / 64 KiB / 256 KiB | {trio('{:.1f}', fe, gb)} | {trio('{:.2f}', fe, km)} ms | "
    f"{trio('{:.3f}', fe, fr)} | {trio('{}', fe, ta)} | {trio('{}', fe, iss)} | — |",
    f"  | consumer verify + decompress, 16 KiB / 64 KiB / 256 KiB (512 MiB) | {trio('{:.1f}', cc, gb)} | "
    f"{trio('{:.2f}', cc, km)} ms | {trio('{:.3f}', cc, fr)} | {trio('{}', cc, ta)} | {trio('{}', cc, iss)} | — |",
    f"  | `configs[0]` workload: 1M × 100 B perf-tool messages, writer + finalize (exact) | {pt['GB_per_s']} "
    f"({pt['msgs_per_s'] / 1e6:.0f} M msgs/s) | {pt['roofline']['kernel_ms']:.2f} ms | {pt['roofline']['frac']} | {ta(pt)} | "
    f"{iss(pt)} | {cpu('perf_tool_1M_x_100B_messages') / 1e6:.1f} M msgs/s |",
    f"  | CRC32C only, 1M × 16 KiB (`configs[1]`) | {c['GB_per_s']:.0f} | {cr['kernel_ms']:.2f} ms / 16 GiB | {cr['frac']:.3f} | "
    f"{round(cr['traffic'] / cr['alg_bytes_per_launch'], 2)} | {(cr.get('issue') or {}).get('frac_of_issue_ceiling')} | "
    f"{cpu('crc32c_only_16KiB_batches'):.0f} (port) |",
    line("compress exact (256 × 1 MiB)", "lz4f_compress_1MiB_json", f"{cpu('lz4f_compress_1MiB_json'):.1f}"),
    line("compress fast", "lz4f_compress_fast_1MiB_json", f"{cpu('lz4f_compress_fast_1MiB_json'):.1f}"),
    line("compress, workgroup-per-block engine (§4.13, ratio 2.823)", "lz4f_compress_units_1MiB_json"),
    line("LZ4HC level 9 (ratio 3.591)", "lz4hc_compress_level9_1MiB_json", f"{cpu('lz4hc_compress_level9_1MiB_json'):.2f}"),
    line("LZ4HC level 12 (ratio 3.634)", "lz4hc_compress_level12_1MiB_json", f"{cpu('lz4hc_compress_level12_1MiB_json'):.2f}"),
    line("snappy compress (ratio 2.665)", "snappy_compress_1MiB_json", f"{cpu('snappy_compress_1MiB_json'):.1f} (port)"),
    line("snappy uncompress (1 GiB)", "snappy_uncompress_1MiB_json", f"{cpu('snappy_uncompress_1MiB_json'):.1f} (port)"),
    line("consumer verify + decompress (1024 × 1 MiB)", "consumer_crc_verify_lz4f_decompress_1MiB",
         f"{cpu('consumer_crc_verify_lz4f_decompress_1MiB'):.1f}"),
    line("record serialise (§4.6)", "v2_record_serialize_1MiB_json", f"{cpu('v2_record_serialize_1MiB_json'):.1f} (1 thr, port)"),
    line("record index (§4.7)", "v2_record_index_1MiB_json", f"{cpu('v2_record_index_1MiB_json'):.1f} (1 thr, port)"),
    line("MsgVersion 1 CRC-32 verify (§4.8)", "v1_msgset_crc32_verify_1MiB_json",
         f"{cpu('v1_msgset_crc32_verify_1MiB_json'):.1f} (1 thr, zlib)"),
    line("whole writer: messages → finished batches (256 × ~0.83 MiB)", "writer_messages_to_batches_1MiB_json"),
    line("whole reader: finished batches → rows", "reader_batches_to_rows_1MiB_json"),
    f"  | producer pipeline, PCIe-inclusive, 1 / 2 / 4 / 8 broker threads | {pp['1_threads']} / {pp['2_threads']} / "
    f"{pp['4_threads']} / {pp['8_threads']} | — | — | — | — | {cpu('producer_pipeline_1MiB_json_pcie'):.1f} |",
]
table = "\n".join(rows) + "\n"
p = os.path.join(ROOT, "DESIGN.md")
s = open(p).read()
a = s.index("| symbol, size | 1 thread | 8 threads, combined |")
b = s.index("One frame is at most 16 blocks = 16 busy waves of a 256-CU chip")
s = s[:a] + dtable + "\n" + s[b:]
a = s.index("  | line | GB/s | kernel time | HBM frac | traffic / alg | issue | CPU reference (16 thr) |")
b = s.index("  The `issue` column is the round's added reading")
s = s[:a] + table + "\n" + s[b:]
open(p, "w").write(s)
print(dtable)
print(table)
