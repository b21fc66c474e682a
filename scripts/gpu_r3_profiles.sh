#!/bin/bash
# rocprofv3 summaries of the bench legs named on the command line (default: all) into
# gpurun_out/prof_r3/summaries/.  Stops at the first leg that fails.
set -o pipefail
P="bash scripts/profile_r3.sh"
run() {
  case "$1" in
    finalize_fast) $P writer_finalize_fast_1MiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel" --workload finalize_fast --steps 10 ;;
    finalize) $P writer_finalize_1MiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload finalize --steps 10 ;;
    finalize_fast_16k) $P writer_finalize_fast_16KiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel,lz4f_max_blocks_kernel" --workload finalize_fast --batch-bytes 16384 --partitions 32768 --steps 10 ;;
    finalize_fast_64k) $P writer_finalize_fast_64KiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel,lz4f_max_blocks_kernel" --workload finalize_fast --batch-bytes 65536 --partitions 8192 --steps 10 ;;
    finalize_fast_256k) $P writer_finalize_fast_256KiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel" --workload finalize_fast --batch-bytes 262144 --partitions 2048 --steps 10 ;;
    finalize_16k) $P writer_finalize_16KiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel,lz4f_max_blocks_kernel" --workload finalize --batch-bytes 16384 --partitions 32768 --steps 10 ;;
    finalize_64k) $P writer_finalize_64KiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel,lz4f_max_blocks_kernel" --workload finalize --batch-bytes 65536 --partitions 8192 --steps 10 ;;
    finalize_256k) $P writer_finalize_256KiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload finalize --batch-bytes 262144 --partitions 2048 --steps 10 ;;
    consumer_16k) $P consumer_crc_verify_lz4f_decompress_16KiB "crc32c_msgset_v2,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel" --workload consumer --batch-bytes 16384 --partitions 32768 --steps 10 ;;
    consumer_64k) $P consumer_crc_verify_lz4f_decompress_64KiB "crc32c_msgset_v2,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel" --workload consumer --batch-bytes 65536 --partitions 8192 --steps 10 ;;
    consumer_256k) $P consumer_crc_verify_lz4f_decompress_256KiB "crc32c_msgset_v2,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel" --workload consumer --batch-bytes 262144 --partitions 2048 --steps 10 ;;
    chain_writer) $P writer_messages_to_batches_1MiB_json "v2_batch_kernel,v2_chunk_kernel,v2_fixup_kernel,v2_write_kernel,lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload chain_writer --partitions 256 --steps 10 ;;
    chain_reader) $P reader_batches_to_rows_1MiB_json "crc32c_msgset_v2,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel,v2_index_spec_kernel,v2_index_kernel" --workload chain_reader --partitions 256 --steps 10 ;;
    crc) $P crc32c_only_16KiB_batches "crc32c_msgset_v2" --workload crc --steps 10 ;;
    lz4c) $P lz4f_compress_1MiB_json "lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4c --partitions 256 --steps 10 ;;
    lz4c_fast) $P lz4f_compress_fast_1MiB_json "lz4_fast_blocks_kernel,lz4f_assemble_kernel" --workload lz4c_fast --partitions 256 --steps 10 ;;
    lz4c_units) $P lz4f_compress_units_1MiB_json "lz4_units_blocks_kernel,lz4f_assemble_kernel" --workload lz4c_units --partitions 256 --steps 10 ;;
    consumer) $P consumer_crc_verify_lz4f_decompress_1MiB "crc32c_msgset_v2,lz4f_walk_kernel,lz4f_blocks_kernel,lz4f_seq_kernel,lz4f_finish_kernel" --workload consumer --partitions 1024 --steps 10 ;;
    lz4hc9) $P lz4hc_compress_level9_1MiB_json "lz4hc_build_kernel,lz4hc_count_items_kernel,lz4hc_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4hc --level 9 --partitions 256 --steps 10 ;;
    lz4hc12) $P lz4hc_compress_level12_1MiB_json "lz4hc_build_kernel,lz4hc_count_items_kernel,lz4hc_compress_blocks_kernel,lz4f_assemble_kernel" --workload lz4hc --level 12 --partitions 256 --steps 10 ;;
    snappyc) $P snappy_compress_1MiB_json "snappy_compress_fragments_kernel,snappy_assemble_kernel" --workload snappyc --partitions 256 --steps 10 ;;
    snappyd) $P snappy_uncompress_1MiB_json "snappy_scan_kernel,snappy_uncompress_kernel" --workload snappyd --partitions 1024 --steps 10 ;;
    serialize) $P v2_record_serialize_1MiB_json "v2_batch_kernel,v2_chunk_kernel,v2_fixup_kernel,v2_write_kernel,crc32c_msgset_v2_split_kernel,crc32c_msgset_v2_combine_kernel" --workload serialize --partitions 256 --steps 10 ;;
    index) $P v2_record_index_1MiB_json "v2_index_spec_kernel,v2_index_kernel" --workload index --partitions 256 --steps 10 ;;
    legacy) $P v1_msgset_crc32_verify_1MiB_json "v01_crc_kernel" --workload legacy --partitions 256 --steps 10 ;;
    perf_tool) $P perf_tool_1M_x_100B_messages "v2_batch_kernel,v2_chunk_kernel,v2_fixup_kernel,v2_write_kernel,lz4_compress_blocks_kernel,lz4f_assemble_kernel" --workload perf_tool --steps 10 ;;
    *) echo "unknown leg $1"; return 1 ;;
  esac
}
LEGS="$*"
[ -n "$LEGS" ] || LEGS="finalize_fast finalize crc lz4c lz4c_fast lz4c_units consumer"
for l in $LEGS; do run "$l" || exit 1; done
ls gpurun_out/prof_r3/summaries
