bash tools/gpu_session.sh \
 "pmck|600|PMC_REGEX=\"k_lines2|k_scan|k_bucket_apply|k_st_claim|k_ip_claim\" VARIANTS=\"r5\" bash tools/pmc_kernel.sh l2 cfg3 20000000"
