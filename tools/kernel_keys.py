"""rocprof kernel name -> bench.py kernel key (the PROF_LAUNCH names of liborbg)."""
KEYS = {
    "k_pyramid": "resize", "k_resize": "resize", "k_fast_cells": "fast_cells", "k_fast2": "fast_cells", "k_fast_rows": "fast_cells",
    "k_blur": "blur", "k_blur2": "blur", "k_blur_border": "blur", "k_octree_lds": "octree", "k_octree": "octree_big",
    "k_orient_desc": "orient_desc", "k_knn2_pairs": "knn2", "k_knn2_pairs_i8": "knn2", "k_init_cands_pairs": "init_cands",
    "k_init_resolve_pairs": "init_resolve", "k_stereo_rows": "stereo_rows",
    "k_stereo_match": "stereo_match", "k_stereo_rows_match": "stereo_match",
    "k_stereo_sad": "stereo_sad", "k_stereo_sad_mg": "stereo_sad",
    "k_stereo_median": "stereo_median", "k_ba_edges": "ba_edges",
    "k_ba_point_blocks": "ba_point_blocks", "k_ba_pose_mfma": "ba_pose_mfma",
    "k_ba_slices_special": "ba_pose_mfma", "k_ba_pose_reduce": "ba_pose_reduce",
    "k_ba_errors": "ba_errors", "k_ba_errors_packed": "ba_errors",
    "k_schur_points": "schur_points", "k_schur_blocks": "schur_blocks",
    "k_schur_blocks_lds": "schur_blocks", "k_schur_rhs": "schur_rhs",
    "k_schur_ldlt": "schur_ldlt", "k_schur_ldlt_wave": "schur_ldlt",
    "k_schur_backsub": "schur_backsub", "k_ba_update": "ba_update", "k_lm_partial": "lm_reduce",
    "k_lm_final": "lm_reduce",
}


def key(kernel_name):
    """'void orbg::k_fast2<12>(...)' -> 'fast_cells' (None for runtime copies)."""
    n = kernel_name.split("(")[0].replace("void ", "").replace("orbg::", "").strip()
    n = n.split("<")[0]
    return KEYS.get(n)
