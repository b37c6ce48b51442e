"""Per-kernel totals of the one-GPU run against each shared-memory rank's (tools/shard_compare.sh
with PROF=1): the D-wide CycleFinder and adjacency kernels of one GPU beside their per-shard
counterparts, and the shard exchange kernels."""
import csv
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_shard"


def load(f):
    out = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Name"])
        n = m.group(1) if m else r["Name"][:40]
        out[n] = out.get(n, 0) + float(r["TotalDurationNs"]) / 1e6
    return out


s = load(f"{d}/single_kernel_stats.csv")
ranks = []
r = 0
while True:
    try:
        ranks.append(load(f"{d}/rank{r}_kernel_stats.csv"))
    except FileNotFoundError:
        break
    r += 1
ONE = {"adjacency": ["k_adjacency_own", "k_own_bounds", "k_dir"],
       "cf_dwide": ["k_post_filter", "k_tips_filter", "k_peel_prep", "k_peel_walk", "k_peel_super", "k_peel_jump",
                    "k_peel_final", "k_peel_branch", "k_peel_apply_list", "k_peel_apply_rulers", "k_popcount",
                    "k_still_valid", "k_peel_init"],
       "searches": ["k_dls", "k_dls_lanes", "k_findcycle"]}
SHARD = {"adjacency": ["k_sdir", "k_adj_queries", "k_adj_answer", "k_adj_store", "k_ones", "k_count_less", "k_run_bounds",
                       "k_adj_ranges"],
         "cf_dwide": ["k_sh_filter", "k_win_req", "k_win_ans", "k_win_apply", "k_flag_msgs", "k_flag_apply", "k_prep",
                      "k_post_bytes", "k_out_win", "k_push_bytes", "k_recv_bytes",
                      "k_bits_list", "k_word_popc64", "k_walk_init", "k_walk", "k_active_rulers", "k_jump_req",
                      "k_jump_ans", "k_jump_apply", "k_jump_cycle", "k_bref_req", "k_bref_ans", "k_bref_req2",
                      "k_res_req", "k_st_ans", "k_res_apply", "k_rm_nonunary", "k_term_req", "k_rm_rulers",
                      "k_set_build", "k_rm_chains", "k_popc", "k_and_words", "k_fill"],
         "regions": ["k_gstart", "k_bfs_seed", "k_bfs_req", "k_bfs_claim", "k_region_list", "k_region_build",
                     "k_region_words"],
         "searches": ["k_dls", "k_dls_lanes", "k_findcycle"],
         "router": ["k_route_count", "k_route_offsets", "k_route_place"]}
print("%-10s %10s %s" % ("group", "one GPU", " ".join("rank%d" % i for i in range(len(ranks)))))
for grp in ["adjacency", "cf_dwide", "regions", "searches", "router"]:
    one = sum(s.get(k, 0) for k in ONE.get(grp, []))
    per = [sum(x.get(k, 0) for k in SHARD[grp]) for x in ranks]
    print("%-10s %10.2f %s" % (grp, one, " ".join("%7.2f" % v for v in per)))
print("\nper-shard kernels (ms, rank 0):")
for k, v in sorted(ranks[0].items(), key=lambda x: -x[1])[:40]:
    print("  %-26s %8.2f" % (k, v))
