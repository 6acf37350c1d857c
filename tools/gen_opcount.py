"""Freezes bench/opcount.json: exact Fp-multiplication counts of every device stage, measured
by running the generic math headers (the code the GPU kernels instantiate) through the
instrumented host build tests/native/hostcheck.hip on one representative set.  One Fp
multiplication = 300 32x32->64 multiply-accumulates (2*12^2 + 12, CIOS), SURVEY.md 8(d)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import blsdata as bd  # noqa: E402

NAMES = ["sig_decode", "sig_subgroup", "pk_decode", "pk_scale", "hash_map", "sig_scale", "miller",
         "g2_add", "fp12_mul", "final_exp", "g1_add", "miller_multi2_per_set", "miller_lines",
         "miller_accum2_per_set", "miller_accum4_per_set"]


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhostcheck.so"))
    lib.hc_opcount.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                               ctypes.POINTER(ctypes.c_ulonglong)]
    pks, m, sig = bd.single_set(1, tag="opcount")
    counts = (ctypes.c_ulonglong * len(NAMES))()
    lib.hc_opcount(sig, pks[0], m, 0xF00DCAFE12345678, counts)
    c = {n: int(counts[i]) for i, n in enumerate(NAMES)}
    # k_miller_fused (lsg_k_miller.hip): items of four pairs; per item the first doubling and
    # bit 62 (P and M phases: 12 + 34 Fp2 products each), 62 further doublings (S, P, M: 12 +
    # 12 + 34) and the additions for the other set bits of |x| (46 each); per set its 68 line
    # steps (miller_lines) and their evaluations at P (two Fp2 x Fp products, 4 Fp products)
    xabs = 0xD201000000010000
    adds = bin(xabs & ((1 << 62) - 1)).count("1")
    fp2_products_per_item = 2 * 46 + 62 * 58 + adds * 46
    c["miller_fused_per_set"] = c["miller_lines"] + 68 * 4 + 3 * fp2_products_per_item // 4
    # device path: multi-Miller items of K = 2 pairs (shared squarings), so per set the Miller
    # stage costs miller_multi2_per_set; one Fp12 product per item in the product tree
    # (the default Miller kernel is k_miller_fused: bench.py swaps miller_multi2_per_set for
    # miller_fused_per_set)
    per_set = (c["sig_decode"] + c["sig_subgroup"] + c["pk_decode"] + c["pk_scale"] + c["hash_map"] + c["sig_scale"]
               + c["miller_multi2_per_set"] + c["g2_add"] + c["fp12_mul"] // 2)
    per_batch = c["miller"] + c["fp12_mul"] + c["final_exp"]  # group sig term + product + FE
    # the device sums sum_i r_i sig_i per group by a bucket MSM (lsg_bls.hip msm_sum: 8-bit
    # windows of the 64-bit r_i) instead of per-set [r_i] sig_i: per set one G2 addition per
    # window digit (8, an upper bound: zero digits are skipped); per group the 64 bit sums over
    # 128 buckets each (64 * 127 additions) and the Horner pass (63 doublings + 63 additions,
    # a doubling counted as an addition)
    msm_per_set = 8 * c["g2_add"]
    msm_per_group = (64 * 127 + 126) * c["g2_add"]
    per_set_msm = per_set - c["sig_scale"] - c["g2_add"] + msm_per_set
    # groups of 32..255 sets: 4-bit windows (lsg_host.hip plan_phase): 16 digits per set, the
    # 64 bit sums over 8 buckets each (64 * 7 additions), the same Horner pass
    msm4_per_set = 16 * c["g2_add"]
    msm4_per_group = (64 * 7 + 126) * c["g2_add"]
    per_set_msm4 = per_set - c["sig_scale"] - c["g2_add"] + msm4_per_set
    # groups of 4..47 sets (16-job chunks, fallback groups): 2-bit windows, 32 digits per set,
    # the 64 bit sums over 2 buckets each (64 additions)
    msm2_per_set = 32 * c["g2_add"]
    msm2_per_group = (64 + 126) * c["g2_add"]
    per_set_msm2 = per_set - c["sig_scale"] - c["g2_add"] + msm2_per_set
    # PublicKey.aggregate of large packages (>= 32768 keys) as the batch-affine tree (lsg_k_pk.hip
    # k_agg_*): per pairwise item 1 prefix product (fold) + 5 (unfold: the item's inverse, the
    # running inverse, lambda, lambda^2, lambda (x1 - x3)); per chunk of 16 items the batched
    # inversion of its product (2 + 1 products and one zero test ~ 1 product per value: 4 / 16)
    # and the zero test of its inverse (1 / 16); a set's last <= 8 points summed with complete
    # mixed additions (11 products; ~7 per set of ~450 keys, spread over its keys)
    tree_per_item = 6 + (4 + 1) / 16
    tree_per_pubkey = round((439 * tree_per_item + 7 * 11) / 446, 2)
    out = {
        "unit": "Fp multiplications (381-bit Montgomery); 1 = 300 v_mad_u64_u32",
        "mads_per_fp_mul": 300,
        "fp2_mul_counting": ("3 Fp products per Fp2 product (the Karatsuba count), whatever leaf computes it: the "
                             "shipped pair leaf (lsg_fp_pair.hpp pair_fp2_mul_sop) runs 4 partial products and 2 "
                             "Montgomery reductions (two sums of products) -- 588 v_mad_i64_i32 per lane, 1,176 per "
                             "lane pair, against 900 in this unit"),
        "stage_fp_muls": c,
        "batched_single_set_fp_muls": per_set,
        "per_batch_fp_muls": per_batch,
        "msm": {"per_set_fp_muls": msm_per_set, "per_group_fp_muls": msm_per_group},
        "batched_single_set_msm_fp_muls": per_set_msm,
        "per_batch_msm_fp_muls": per_batch + msm_per_group,
        "msm2": {"per_set_fp_muls": msm2_per_set, "per_group_fp_muls": msm2_per_group},
        "batched_single_set_msm2_fp_muls": per_set_msm2,
        "per_batch_msm2_fp_muls": per_batch + msm2_per_group,
        "msm4": {"per_set_fp_muls": msm4_per_set, "per_group_fp_muls": msm4_per_group},
        "batched_single_set_msm4_fp_muls": per_set_msm4,
        "per_batch_msm4_fp_muls": per_batch + msm4_per_group,
        "aggregate_extra_per_pubkey_fp_muls": c["g1_add"],
        "aggregate_tree_extra_per_pubkey_fp_muls": tree_per_pubkey,
        "survey_estimate_blst_equivalent": {"batched_single_set": 16000, "per_batch": 15000, "per_pubkey": 11},
        "source": "tools/gen_opcount.py over tests/native/hostcheck.hip (LSG_COUNT_MULS)",
    }
    json.dump(out, open(os.path.join(ROOT, "bench", "opcount.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
