# Every profiled leg of the bench line (copy gpurun_out/prof_r2/summaries/* to profiles/r02/).
set -o pipefail
R="$GRAFT_REPO_ROOT"; P="$R/scripts/profile_r2.sh"
bash $P writer_finalize_1MiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel" --steps 5 --warmup 1 &&
bash $P writer_finalize_fast_1MiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel" --workload finalize_fast --partitions 256 --steps 3 --warmup 1 &&
bash $P crc32c_only_16KiB_batches "crc32c_msgset_v2_v4_kernel" --workload crc --steps 10 --warmup 2 &&
bash $P lz4f_compress_1MiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4c --partitions 256 --steps 3 --warmup 1 &&
bash $P lz4f_compress_fast_1MiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel" --workload lz4c_fast --partitions 256 --steps 3 --warmup 1 &&
bash $P lz4hc_compress_level9_1MiB_json "lz4hc_build_kernel,lz4hc_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4hc --partitions 256 --steps 3 --warmup 1 &&
bash $P lz4hc_compress_level12_1MiB_json "lz4hc_build_kernel,lz4hc_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4hc --level 12 --partitions 256 --steps 2 --warmup 1 &&
bash $P snappy_compress_1MiB_json "snappy_compress_fragments_kernel,snappy_assemble_kernel" --workload snappyc --partitions 256 --steps 3 --warmup 1 &&
bash $P snappy_uncompress_1MiB_json "snappy_scan_kernel,snappy_uncompress_kernel" --workload snappyd --partitions 1024 --steps 3 --warmup 1 &&
bash $P consumer_crc_verify_lz4f_decompress_1MiB "crc32c_msgset_v2_split_kernel,crc32c_msgset_v2_combine_kernel,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel" --workload consumer --partitions 1024 --steps 3 --warmup 1 &&
bash $P v2_record_serialize_1MiB_json "v2_chunk_kernel,v2_batch_kernel,v2_fixup_kernel,v2_write_kernel" --workload serialize --partitions 256 --steps 5 --warmup 1 &&
bash $P v2_record_index_1MiB_json "v2_index_spec_kernel" --workload index --partitions 256 --steps 5 --warmup 1 &&
echo PROFILE_ALL_OK
