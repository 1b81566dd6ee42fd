#!/usr/bin/env python3
"""Freeze the algorithmic work model of the engine's per-item schedule.

Builds the host copy of the device math with TBG_COUNT_OPS (every Montgomery
product / square / reduction adds its u32 multiply-add count) and measures
one item of each pipeline stage on real inputs from the golden fixtures.
Writes profiles/work_model.json, which bench.py uses for roofline.achieved.
One Fp multiplication = 392 u32 mul-adds in this radix-2^28 schedule
(196 a*b + 196 m*p); the survey's 12x32-bit CIOS figure is 300.
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tests", "hostcheck", "hostcheck.cpp")
LIB = os.path.join(ROOT, "tests", "hostcheck", "libhostcheck_count.so")


def main():
    subprocess.check_call(["/opt/rocm/llvm/bin/clang++", "-O1", "-std=c++17", "-fPIC", "-shared", "-DTBG_COUNT_OPS",
                           "-Wno-pass-failed", SRC, "-o", LIB])
    lib = ctypes.CDLL(LIB)
    lib.hc_count_get.restype = ctypes.c_ulonglong
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "cfg1_3of4_single.json")))["vectors"][0]
    msg = bytes.fromhex(gold["msg"])
    sigs = [bytes.fromhex(p["sig"]) for p in gold["partials"]]
    pks = [bytes.fromhex(gold["tss"]["pubshares"][str(p["identifier"])]) for p in gold["partials"]]

    def measure(fn, *a):
        lib.hc_count_reset()
        r = fn(*a)
        return lib.hc_count_get(), r

    decode, st = measure(lib.hc_stage_decode_sig, sigs[0])
    assert st == 0
    hash_, _ = measure(lib.hc_stage_hash, msg, len(msg))
    lib.hc_count_reset()
    assert lib.hc_stage_verify(pks[0], sigs[0], msg, len(msg)) == 1
    verify = lib.hc_count_get()
    lib.hc_count_reset()
    assert lib.hc_stage_lines(sigs[0], msg, len(msg)) == 0
    lines_sig = lib.hc_count_get()
    # H lines alone (per message): total of both minus the signature share
    lib.hc_count_reset()
    lib.hc_stage_lines(sigs[0], msg, len(msg))
    # same schedule (68 steps on a G2 point) without folding P in: k_lines_h
    # stores l1, l4 unevaluated (bls_pair.h EVAL = false), two Fp2 x Fp
    # products (4 Fp products) fewer per line
    lines_h = lines_sig - 68 * 4 * 392
    lib.hc_count_reset()
    assert lib.hc_stage_verify_quad(pks[0]) == 1
    verify_quad = lib.hc_count_get()
    out = ctypes.create_string_buffer(96)
    ids = bytes([p["identifier"] for p in gold["partials"]])
    lib.hc_count_reset()
    assert lib.hc_stage_aggregate(ids, b"".join(sigs), len(sigs), out) == 0
    agg_with_decode = lib.hc_count_get()
    assert out.raw.hex() == gold["expect"]["agg"]
    agg = agg_with_decode - len(sigs) * decode
    # RLC schedule (k_rlc.hip), default group G = 16 duties, chunk C = 4 duties
    G, C = 16, 4
    for fn in ("hc_stage_setup", "hc_stage_rlc_partial", "hc_stage_duty_sum", "hc_stage_group_lines",
               "hc_stage_miller_chunk", "hc_stage_group_final"):
        getattr(lib, fn).restype = ctypes.c_int
    lib.hc_stage_rlc_partial.argtypes = [ctypes.c_uint64]
    assert lib.hc_stage_setup(sigs[0], pks[0], msg, len(msg)) == 0
    rlc_partial, _ = measure(lib.hc_stage_rlc_partial, 0x9E3779B97F4A7C15)
    duty_sum4, _ = measure(lib.hc_stage_duty_sum, 4)
    group_lines8, _ = measure(lib.hc_stage_group_lines, G)
    chunk2, _ = measure(lib.hc_stage_miller_chunk, C, 0)
    chunk2f, _ = measure(lib.hc_stage_miller_chunk, C, 1)
    final4, _ = measure(lib.hc_stage_group_final, G // C)
    rlc_check_per_group = chunk2f + (G // C - 1) * chunk2 + final4
    # Level 0 (k_msm.hip): per partial the G1 table product and 4 bucket
    # additions; per duty the G1-only sum; per group its P chunks and the
    # products folding them (nch quad products, tree included); per launch
    # the bucket scalings (sampled over j), the tree sums, S's lines, S's
    # Miller quad and ONE final exponentiation.
    for fn in ("hc_stage_l0_partial", "hc_stage_duty_sum_p", "hc_stage_l0_bucket_scale", "hc_stage_g2_add"):
        getattr(lib, fn).restype = None
    lib.hc_stage_l0_partial.argtypes = [ctypes.c_uint64]
    lib.hc_stage_l0_bucket_scale.argtypes = [ctypes.c_uint32]
    l0_partial, _ = measure(lib.hc_stage_l0_partial, 0x9E3779B97F4A7C15)
    duty_sum_p4, _ = measure(lib.hc_stage_duty_sum_p, 4)
    step = 61
    scale_sample = [measure(lib.hc_stage_l0_bucket_scale, 2 * j + 1)[0] for j in range(0, 32768, step)]
    bucket_scales = sum(scale_sample) * 32768 / len(scale_sample)
    g2_add, _ = measure(lib.hc_stage_g2_add)
    final1, _ = measure(lib.hc_stage_group_final, 1)
    qmul = measure(lib.hc_stage_group_final, 2)[0] - final1
    s_quad, _ = measure(lib.hc_stage_miller_chunk, 0, 1)
    nch = G // C
    # a P-chunk hexad of c duties costs base + c * per_duty (62 squarings, 68
    # line products per duty): the level-0 launch shape (G, C) varies with the
    # launch size (tbls_engine.hip l0_shape), so the kernels' models are per
    # chunk and per duty
    chunk8, _ = measure(lib.hc_stage_miller_chunk, 8, 0)
    chunk_per_duty = (chunk8 - chunk2) / 4
    chunk_base = chunk2 - 4 * chunk_per_duty
    # per-kernel probes (one item of each kernel of the level-0 chain)
    for fn in ("hc_k_decode_sigs", "hc_k_subgroup_sigs"):
        getattr(lib, fn).restype = ctypes.c_int
    for fn in ("hc_k_hash_map", "hc_k_hash_sswu", "hc_k_hash_clear_setup", "hc_k_hash_clear_x1", "hc_k_hash_clear_x2",
               "hc_k_hash_clear_fin", "hc_k_g2_affine", "hc_k_rlc_g1_l0", "hc_k_msm_entry"):
        getattr(lib, fn).restype = None
    lib.hc_k_rlc_g1_l0.argtypes = [ctypes.c_uint64]
    lib.hc_k_msm_entry.argtypes = [ctypes.c_uint32]
    k_decode, st = measure(lib.hc_k_decode_sigs, sigs[0])
    assert st == 0
    k_subgroup, st = measure(lib.hc_k_subgroup_sigs, sigs[0])
    assert st == 1
    k_hash_map, _ = measure(lib.hc_k_hash_map, msg, len(msg))
    k_hash_sswu, _ = measure(lib.hc_k_hash_sswu)
    lib.hc_k_hash_clear_setup(msg, len(msg))
    k_clear_x1, _ = measure(lib.hc_k_hash_clear_x1)
    k_clear_x2, _ = measure(lib.hc_k_hash_clear_x2)
    k_clear_fin, _ = measure(lib.hc_k_hash_clear_fin)
    k_g2_aff, _ = measure(lib.hc_k_g2_affine)
    k_g1_l0, _ = measure(lib.hc_k_rlc_g1_l0, 0x9E3779B97F4A7C15)
    k_msm_entry = sum(measure(lib.hc_k_msm_entry, k)[0] for k in range(4)) / 4
    # Montgomery's trick over a workgroup (bls_batchinv.h): its per-value cost
    # replaces one fp_inv in every batched kernel (k_hash_map's SSWU
    # denominator, k_hash_affine, k_rlc_duty_sum, k_aggregate)
    for fn in ("hc_fp_inv_once", "hc_batch_inv_cost"):
        getattr(lib, fn).restype = None
    lib.hc_batch_inv_cost.argtypes = [ctypes.c_int, ctypes.c_int]
    fp_inv_cost, _ = measure(lib.hc_fp_inv_once)
    binv_n = 256 * 8
    binv_item = measure(lib.hc_batch_inv_cost, binv_n, 4)[0] / binv_n
    saved = fp_inv_cost - binv_item  # per batched inversion
    k_hash_map -= saved
    k_g2_aff -= saved
    agg -= saved
    duty_sum_p4 -= saved
    duty_sum4 -= saved
    rlc_partial -= saved  # (k_rlc_partial2: the n2 inversion batched; its G1 product now from the key's table)
    hash_ -= 2 * saved
    # batched subgroup test (k_sgb.hip, SGB_M = 1024, 18 combinations with
    # digits uniform mod 13: 12/13 of them non-zero): per partial 18 * 12 / 13
    # mixed additions into buckets; per group and combination the running
    # sums over 6 buckets x 4 slices (30 additions) and one psi(Q) == [x]Q
    # test on a Jacobian Q (the affine test with its 5 mixed additions full)
    madd, _ = measure(lib.hc_k_msm_entry, 0)  # k = 0: psi^0, one mixed addition
    sgb_m, sgb_k = 1024, 18
    sgb_bucket = sgb_k * 12 / 13 * madd
    sgb_fold = sgb_k * 6 * 3 * g2_add / sgb_m  # each bucket's 4 slices into one
    sgb_combine = sgb_k * 12 * g2_add / sgb_m  # the running sums over the 6 folded buckets
    sgb_test = sgb_k * (k_subgroup + 5 * (g2_add - madd)) / sgb_m
    sgb_per_partial = sgb_bucket + sgb_fold + sgb_combine + sgb_test
    decode_sgb = k_decode + sgb_per_partial
    l0_per_group = nch * chunk2 + nch * qmul
    l0_per_launch = bucket_scales + (32768 + 2048 + 128 + 8) * g2_add + lines_h + s_quad + final1
    launch_dvs = 16 * 10000  # bench default: 16 batches of 10k DVs per launch
    unit_3of4_l0_alone = (4 * decode + hash_ + lines_h + 4 * l0_partial + duty_sum_p4 + l0_per_group / G + agg
                          + l0_per_launch / launch_dvs)
    # the default chain: decode + the batched subgroup test instead of one
    # subgroup test per signature
    unit_3of4_l0 = unit_3of4_l0_alone - 4 * decode + 4 * decode_sgb
    # every candidate but the first of each group is randomised: (4 G - 1) / G per duty
    unit_3of4_rlc = (4 * decode + hash_ + lines_h + (4 * G - 1) / G * rlc_partial + duty_sum4 + group_lines8 / G
                     + rlc_check_per_group / G + agg)
    unit_3of4_v1 = 4 * decode + hash_ + 4 * verify + agg
    unit_3of4 = 4 * decode + hash_ + lines_h + 4 * (lines_sig + verify_quad) + agg
    model = {
        "generator": "tools/count_work.py",
        "mads_per_fp_mul": 392,
        "rlc_schedule": {"group": G, "chunk": C},
        "mads": {"decode_sig": decode, "hash_to_g2": hash_, "lines_sig": lines_sig, "lines_h": lines_h,
                 "verify_quad_item": verify_quad, "verify_item_single_lane": verify,
                 "rlc_partial": rlc_partial, "rlc_duty_sum_4": duty_sum4, "rlc_group_lines": group_lines8,
                 "rlc_miller_chunk": chunk2, "rlc_miller_chunk_folded": chunk2f, "rlc_group_final": final4,
                 "rlc_check_per_group": rlc_check_per_group,
                 "aggregate_3of4_all4": agg,
                 "l0_partial": l0_partial, "l0_duty_sum_4": duty_sum_p4, "l0_per_group": l0_per_group,
                 "l0_per_launch": round(l0_per_launch), "l0_bucket_scales": round(bucket_scales),
                 "g2_add": g2_add, "quad_mul": qmul, "l0_s_quad": s_quad, "final_exp_quad": final1,
                 "l0_chunk_base": round(chunk_base), "l0_chunk_per_duty": round(chunk_per_duty),
                 "unit_3of4_l0": round(unit_3of4_l0), "l0_launch_dvs": launch_dvs,
                 "unit_3of4_l0_subgroup_alone": round(unit_3of4_l0_alone),
                 "decode_sig_batched_subgroup": round(decode_sgb), "sgb_per_partial": round(sgb_per_partial),
                 "unit_3of4_rlc": round(unit_3of4_rlc), "unit_3of4_each": unit_3of4,
                 "unit_3of4_single_lane_schedule": unit_3of4_v1},
        "fp_mul_equiv": {k: round(v / 392, 1) for k, v in
                         {"decode_sig": decode, "hash_to_g2": hash_, "lines_sig": lines_sig,
                          "verify_quad_item": verify_quad, "verify_item_single_lane": verify,
                          "rlc_partial": rlc_partial, "rlc_duty_sum_4": duty_sum4,
                          "rlc_group_lines": group_lines8, "rlc_miller_chunk": chunk2,
                          "rlc_miller_chunk_folded": chunk2f, "rlc_group_final": final4,
                          "aggregate_3of4_all4": agg, "l0_partial": l0_partial, "l0_duty_sum_4": duty_sum_p4,
                          "l0_per_group": l0_per_group, "l0_per_launch": l0_per_launch,
                          "unit_3of4_l0": unit_3of4_l0, "unit_3of4_rlc": unit_3of4_rlc,
                          "decode_sig_batched_subgroup": decode_sgb,
                          "unit_3of4_each": unit_3of4, "unit_3of4_reference_schedule": unit_3of4_v1}.items()},
        "verify_hbm_bytes_per_launch": None,
        "batched_inversion": {"fp_inv": fp_inv_cost, "per_value_in_workgroups_of_256": round(binv_item, 1)},
        # u32 mul-adds per item of each kernel of the level-0 chain (bench.py
        # prices the dominant kernel of its per-kernel profile with these)
        "kernels": {
            "k_decode_sigs": {"per": "partial", "mads": round(k_decode)},
            "k_subgroup_sigs": {"per": "partial", "mads": round(k_subgroup)},
            "k_sgb_bucket": {"per": "partial", "mads": round(sgb_bucket)},
            "k_sgb_fold": {"per": "partial", "mads": round(sgb_fold)},
            "k_sgb_combine": {"per": "partial", "mads": round(sgb_combine)},
            "k_sgb_test": {"per": "partial", "mads": round(sgb_test)},
            "k_hash_map": {"per": "message", "mads": round(k_hash_map)},
            "k_hash_sswu": {"per": "message", "mads": round(k_hash_sswu)},
            "k_hash_clear_x1": {"per": "message", "mads": round(k_clear_x1)},
            "k_hash_clear_x2": {"per": "message", "mads": round(k_clear_x2)},
            "k_hash_clear_fin": {"per": "message", "mads": round(k_clear_fin)},
            "k_hash_affine": {"per": "message", "mads": round(k_g2_aff)},
            "k_lines_h": {"per": "message", "mads": round(lines_h)},
            "k_rlc_g1_l0": {"per": "partial", "mads": round(k_g1_l0)},
            "k_msm_bucket_part": {"per": "partial", "mads": round(4 * k_msm_entry)},
            "k_msm_bucket": {"per": "launch", "mads": round(bucket_scales + 32768 * (4 - 1) * g2_add)},
            "k_rlc_duty_sum<DSUM_L0_P>": {"per": "duty", "mads": round(duty_sum_p4)},
            # the level-0 P-chunk products on hexads (bls_hex.h) + the one S hexad
            "k_miller_hex<MILLER_L0>": {"per": "chunk", "mads": round(chunk_base), "plus": {"duty": round(chunk_per_duty)},
                                        "plus_per_launch": s_quad},
            "k_l0_fold": {"per": "chunk", "mads": round(qmul), "plus": {"group": -round(qmul)}},
            "k_l0_final": {"per": "launch", "mads": round(final1)},
            "k_aggregate<true>": {"per": "duty", "mads": round(agg)},
            "k_aggregate<false>": {"per": "duty", "mads": round(agg)},
        },
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "work_model.json"), "w") as f:
        json.dump(model, f, indent=1)
    print(json.dumps(model, indent=1))


if __name__ == "__main__":
    main()
