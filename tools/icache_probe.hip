#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define BODY asm volatile("s_mov_b32 s40, 0xfffaaab\ns_mov_b32 s41, 0xfefffff\ns_mov_b32 s42, 0x3ffffb9\ns_mov_b32 s43, 0xfffeb15\ns_mov_b32 s44, 0x6241eab\ns_mov_b32 s45, 0xa0f6b0f\ns_mov_b32 s46, 0xf6730d2\ns_mov_b32 s47, 0xf38512b\ns_mov_b32 s48, 0x4774b84\ns_mov_b32 s49, 0x4bacd76\ns_mov_b32 s50, 0xba7b643\ns_mov_b32 s51, 0xe69a4b1\ns_mov_b32 s52, 0x1ea397f\ns_mov_b32 s53, 0x1a011\ns_mov_b32 s54, 0xffcfffd\nv_mad_u64_u32 v[42:43], vcc, v0, v14, 0\nv_mul_lo_u32 v44, v42, s54\nv_and_b32 v44, 0xfffffff, v44\nv_mad_u64_u32 v[42:43], vcc, v44, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s41, v[42:43]\nv_mul_lo_u32 v45, v42, s54\nv_and_b32 v45, 0xfffffff, v45\nv_mad_u64_u32 v[42:43], vcc, v45, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s41, v[42:43]\nv_mul_lo_u32 v46, v42, s54\nv_and_b32 v46, 0xfffffff, v46\nv_mad_u64_u32 v[42:43], vcc, v46, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s41, v[42:43]\nv_mul_lo_u32 v47, v42, s54\nv_and_b32 v47, 0xfffffff, v47\nv_mad_u64_u32 v[42:43], vcc, v47, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s41, v[42:43]\nv_mul_lo_u32 v48, v42, s54\nv_and_b32 v48, 0xfffffff, v48\nv_mad_u64_u32 v[42:43], vcc, v48, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s41, v[42:43]\nv_mul_lo_u32 v49, v42, s54\nv_and_b32 v49, 0xfffffff, v49\nv_mad_u64_u32 v[42:43], vcc, v49, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s41, v[42:43]\nv_mul_lo_u32 v50, v42, s54\nv_and_b32 v50, 0xfffffff, v50\nv_mad_u64_u32 v[42:43], vcc, v50, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s41, v[42:43]\nv_mul_lo_u32 v51, v42, s54\nv_and_b32 v51, 0xfffffff, v51\nv_mad_u64_u32 v[42:43], vcc, v51, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s41, v[42:43]\nv_mul_lo_u32 v52, v42, s54\nv_and_b32 v52, 0xfffffff, v52\nv_mad_u64_u32 v[42:43], vcc, v52, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s41, v[42:43]\nv_mul_lo_u32 v53, v42, s54\nv_and_b32 v53, 0xfffffff, v53\nv_mad_u64_u32 v[42:43], vcc, v53, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s41, v[42:43]\nv_mul_lo_u32 v54, v42, s54\nv_and_b32 v54, 0xfffffff, v54\nv_mad_u64_u32 v[42:43], vcc, v54, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s41, v[42:43]\nv_mul_lo_u32 v55, v42, s54\nv_and_b32 v55, 0xfffffff, v55\nv_mad_u64_u32 v[42:43], vcc, v55, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s41, v[42:43]\nv_mul_lo_u32 v56, v42, s54\nv_and_b32 v56, 0xfffffff, v56\nv_mad_u64_u32 v[42:43], vcc, v56, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v0, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v14, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v44, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s41, v[42:43]\nv_mul_lo_u32 v57, v42, s54\nv_and_b32 v57, 0xfffffff, v57\nv_mad_u64_u32 v[42:43], vcc, v57, s40, v[42:43]\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v1, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v15, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v45, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s42, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s41, v[42:43]\nv_and_b32 v28, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v2, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v16, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v46, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s43, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s42, v[42:43]\nv_and_b32 v29, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v3, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v17, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v47, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s44, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s43, v[42:43]\nv_and_b32 v30, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v4, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v18, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v48, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s45, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s44, v[42:43]\nv_and_b32 v31, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v5, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v19, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v49, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s46, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s45, v[42:43]\nv_and_b32 v32, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v6, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v20, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v50, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s47, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s46, v[42:43]\nv_and_b32 v33, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v7, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v21, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v51, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s48, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s47, v[42:43]\nv_and_b32 v34, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v8, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v22, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v52, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s49, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s48, v[42:43]\nv_and_b32 v35, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v9, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v23, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v53, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s50, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s49, v[42:43]\nv_and_b32 v36, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v10, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v24, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v54, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s51, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s50, v[42:43]\nv_and_b32 v37, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v11, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v25, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v55, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s52, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s51, v[42:43]\nv_and_b32 v38, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v12, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v26, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v56, s53, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s52, v[42:43]\nv_and_b32 v39, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v13, v27, v[42:43]\nv_mad_u64_u32 v[42:43], vcc, v57, s53, v[42:43]\nv_and_b32 v40, 0xfffffff, v42\nv_lshrrev_b64 v[42:43], 28, v[42:43]\nv_mov_b32 v41, v42" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "vcc");
__global__ void __launch_bounds__(64) k1(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
__global__ void __launch_bounds__(64) k4(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
    BODY
    BODY
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
__global__ void __launch_bounds__(64) k8(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
__global__ void __launch_bounds__(64) k16(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
__global__ void __launch_bounds__(64) k32(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
__global__ void __launch_bounds__(64) k64(uint32_t* out, int iters) {
  for (int it = 0; it < iters; it++) {
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
    BODY
  }
  if (iters < 0) out[threadIdx.x] = 1;
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 4096); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  k1<<<1024 * 1, 64>>>(d, 512); (void)hipEventRecord(e0); k1<<<1024 * 1, 64>>>(d, 512); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 1, 1 * 3.8, ms, ms * 1e6 / 512 / 1);
  k4<<<1024 * 1, 64>>>(d, 128); (void)hipEventRecord(e0); k4<<<1024 * 1, 64>>>(d, 128); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 4, 4 * 3.8, ms, ms * 1e6 / 512 / 1);
  k8<<<1024 * 1, 64>>>(d, 64); (void)hipEventRecord(e0); k8<<<1024 * 1, 64>>>(d, 64); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 8, 8 * 3.8, ms, ms * 1e6 / 512 / 1);
  k16<<<1024 * 1, 64>>>(d, 32); (void)hipEventRecord(e0); k16<<<1024 * 1, 64>>>(d, 32); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 16, 16 * 3.8, ms, ms * 1e6 / 512 / 1);
  k32<<<1024 * 1, 64>>>(d, 16); (void)hipEventRecord(e0); k32<<<1024 * 1, 64>>>(d, 16); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 32, 32 * 3.8, ms, ms * 1e6 / 512 / 1);
  k64<<<1024 * 1, 64>>>(d, 8); (void)hipEventRecord(e0); k64<<<1024 * 1, 64>>>(d, 8); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=1 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 64, 64 * 3.8, ms, ms * 1e6 / 512 / 1);
  k1<<<1024 * 2, 64>>>(d, 512); (void)hipEventRecord(e0); k1<<<1024 * 2, 64>>>(d, 512); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 1, 1 * 3.8, ms, ms * 1e6 / 512 / 2);
  k4<<<1024 * 2, 64>>>(d, 128); (void)hipEventRecord(e0); k4<<<1024 * 2, 64>>>(d, 128); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 4, 4 * 3.8, ms, ms * 1e6 / 512 / 2);
  k8<<<1024 * 2, 64>>>(d, 64); (void)hipEventRecord(e0); k8<<<1024 * 2, 64>>>(d, 64); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 8, 8 * 3.8, ms, ms * 1e6 / 512 / 2);
  k16<<<1024 * 2, 64>>>(d, 32); (void)hipEventRecord(e0); k16<<<1024 * 2, 64>>>(d, 32); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 16, 16 * 3.8, ms, ms * 1e6 / 512 / 2);
  k32<<<1024 * 2, 64>>>(d, 16); (void)hipEventRecord(e0); k32<<<1024 * 2, 64>>>(d, 16); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 32, 32 * 3.8, ms, ms * 1e6 / 512 / 2);
  k64<<<1024 * 2, 64>>>(d, 8); (void)hipEventRecord(e0); k64<<<1024 * 2, 64>>>(d, 8); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=2 K=%3d body %7.1f KB: %8.3f ms, %.1f ns per product per SIMD\n", 64, 64 * 3.8, ms, ms * 1e6 / 512 / 2);
  return 0; }
