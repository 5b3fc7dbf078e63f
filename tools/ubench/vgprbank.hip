// vgprbank.hip -- does VGPR bank placement of VOP3 sources cost issue cycles on
// gfx950?  Same 24-instruction independent streams, sources in distinct banks
// (reg % 4 all different) vs all in one bank.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"

// distinct banks: dst v40+i, srcs v(41), v(42), v(43) pattern -> banks 1,2,3
#define DB(op) op " v40, v41, v42, v43\n\t" op " v44, v45, v46, v47\n\t" op " v48, v49, v50, v51\n\t" op " v52, v53, v54, v55\n\t" \
               op " v56, v57, v58, v59\n\t" op " v60, v61, v62, v63\n\t"
// same bank: srcs all == 1 mod 4
#define SB(op) op " v40, v41, v45, v49\n\t" op " v44, v53, v57, v61\n\t" op " v48, v41, v45, v49\n\t" op " v52, v53, v57, v61\n\t" \
               op " v56, v41, v45, v49\n\t" op " v60, v53, v57, v61\n\t"

#define L64(op) op " v[40:41], v[42:43], 5, v[44:45]\n\t" op " v[46:47], v[48:49], 5, v[50:51]\n\t" op " v[52:53], v[54:55], 5, v[56:57]\n\t" \
               op " v[58:59], v[60:61], 5, v[62:63]\n\t" op " v[40:41], v[48:49], 5, v[56:57]\n\t" op " v[46:47], v[54:55], 5, v[62:63]\n\t"
#define SH64(op) op " v[40:41], 5, v[42:43]\n\t" op " v[44:45], 5, v[46:47]\n\t" op " v[48:49], 5, v[50:51]\n\t" \
               op " v[52:53], 5, v[54:55]\n\t" op " v[56:57], 5, v[58:59]\n\t" op " v[60:61], 5, v[62:63]\n\t"
#define PKMOV(op) op " v[40:41], v[42:43], v[44:45] op_sel:[1,0]\n\t" op " v[46:47], v[48:49], v[50:51] op_sel:[1,0]\n\t" op " v[52:53], v[54:55], v[56:57] op_sel:[1,0]\n\t" \
               op " v[58:59], v[60:61], v[62:63] op_sel:[1,0]\n\t" op " v[40:41], v[48:49], v[56:57] op_sel:[1,0]\n\t" op " v[46:47], v[54:55], v[62:63] op_sel:[1,0]\n\t"
// the rotate form the SHA-1 rounds use: both data sources the same register, constant shift
#define ROT(n) "v_alignbit_b32 v40, v41, v41, " #n "\n\tv_alignbit_b32 v44, v45, v45, " #n "\n\tv_alignbit_b32 v48, v49, v49, " #n "\n\t" \
               "v_alignbit_b32 v52, v53, v53, " #n "\n\tv_alignbit_b32 v56, v57, v57, " #n "\n\tv_alignbit_b32 v60, v61, v61, " #n "\n\t"
// two of three sources in one bank (v41/v45/v49/v53/v57/v61 are bank 1; v42.. bank 2)
#define SB2(op) op " v40, v41, v45, v42\n\t" op " v44, v49, v53, v46\n\t" op " v48, v57, v61, v50\n\t" op " v52, v41, v49, v54\n\t" \
                op " v56, v45, v53, v58\n\t" op " v60, v57, v41, v62\n\t"
// two-source VOP2: same bank vs distinct banks
#define X2S(op) op " v40, v41, v45\n\t" op " v44, v49, v53\n\t" op " v48, v57, v61\n\t" op " v52, v41, v49\n\t" op " v56, v45, v53\n\t" op " v60, v57, v41\n\t"
#define X2D(op) op " v40, v41, v42\n\t" op " v44, v45, v46\n\t" op " v48, v49, v50\n\t" op " v52, v53, v54\n\t" op " v56, v57, v58\n\t" op " v60, v61, v62\n\t"
#define MOV(op) op " v40, v41\n\t" op " v44, v45\n\t" op " v48, v49\n\t" op " v52, v53\n\t" op " v56, v57\n\t" op " v60, v61\n\t"
#define ADDCO(op) op " v40, vcc, v41, v42\n\t" op " v44, vcc, v45, v46\n\t" op " v48, vcc, v49, v50\n\t" op " v52, vcc, v53, v54\n\t" op " v56, vcc, v57, v58\n\t" op " v60, vcc, v61, v62\n\t"

template <int P>
__global__ __launch_bounds__(256) void kern(uint32_t *out, int iters) {
  asm volatile("v_mov_b32 v41, 1\n\tv_mov_b32 v42, 2\n\tv_mov_b32 v43, 3\n\tv_mov_b32 v45, 5\n\tv_mov_b32 v46, 6\n\tv_mov_b32 v47, 7\n\t"
               "v_mov_b32 v49, 9\n\tv_mov_b32 v50, 10\n\tv_mov_b32 v51, 11\n\tv_mov_b32 v53, 13\n\tv_mov_b32 v54, 14\n\tv_mov_b32 v55, 15\n\t"
               "v_mov_b32 v57, 17\n\tv_mov_b32 v58, 18\n\tv_mov_b32 v59, 19\n\tv_mov_b32 v61, 21\n\tv_mov_b32 v62, 22\n\tv_mov_b32 v63, 23" ::: CLOB);
  for (int it = 0; it < iters; ++it) {
    if constexpr (P == 0) asm volatile(DB("v_add3_u32") DB("v_add3_u32") DB("v_add3_u32") DB("v_add3_u32") ::: CLOB);
    if constexpr (P == 1) asm volatile(SB("v_add3_u32") SB("v_add3_u32") SB("v_add3_u32") SB("v_add3_u32") ::: CLOB);
    if constexpr (P == 2) asm volatile(DB("v_bitop3_b32") DB("v_bitop3_b32") DB("v_bitop3_b32") DB("v_bitop3_b32") ::: CLOB);
    if constexpr (P == 3) asm volatile(SB("v_bitop3_b32") SB("v_bitop3_b32") SB("v_bitop3_b32") SB("v_bitop3_b32") ::: CLOB);
    if constexpr (P == 4) asm volatile(DB("v_alignbit_b32") DB("v_alignbit_b32") DB("v_alignbit_b32") DB("v_alignbit_b32") ::: CLOB);
    if constexpr (P == 6) asm volatile(L64("v_lshl_add_u64") L64("v_lshl_add_u64") L64("v_lshl_add_u64") L64("v_lshl_add_u64") ::: CLOB);
    if constexpr (P == 7) asm volatile(SH64("v_lshlrev_b64") SH64("v_lshlrev_b64") SH64("v_lshlrev_b64") SH64("v_lshlrev_b64") ::: CLOB);
    if constexpr (P == 8) asm volatile(PKMOV("v_pk_mov_b32") PKMOV("v_pk_mov_b32") PKMOV("v_pk_mov_b32") PKMOV("v_pk_mov_b32") ::: CLOB);
    if constexpr (P == 9) asm volatile(MOV("v_mov_b32") MOV("v_mov_b32") MOV("v_mov_b32") MOV("v_mov_b32") ::: CLOB);
    if constexpr (P == 10) asm volatile(ADDCO("v_add_co_u32") ADDCO("v_add_co_u32") ADDCO("v_add_co_u32") ADDCO("v_add_co_u32") ::: CLOB, "vcc");
    if constexpr (P == 5) asm volatile(SB("v_alignbit_b32") SB("v_alignbit_b32") SB("v_alignbit_b32") SB("v_alignbit_b32") ::: CLOB);
    if constexpr (P == 12) asm volatile(SB2("v_bitop3_b32") SB2("v_bitop3_b32") SB2("v_bitop3_b32") SB2("v_bitop3_b32") ::: CLOB);
    if constexpr (P == 13) asm volatile(X2S("v_xor_b32") X2S("v_xor_b32") X2S("v_xor_b32") X2S("v_xor_b32") ::: CLOB);
    if constexpr (P == 14) asm volatile(X2D("v_xor_b32") X2D("v_xor_b32") X2D("v_xor_b32") X2D("v_xor_b32") ::: CLOB);
    if constexpr (P == 11) asm volatile(ROT(27) ROT(2) ROT(31) ROT(27) ::: CLOB);
  }
  uint32_t r;
  asm volatile("v_xor_b32 %0, v40, v44\n\tv_xor_b32 %0, %0, v48" : "=v"(r) :: CLOB);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int P>
void run(const char *name, int w) {
  const int blocks = 256 * w, iters = 20000;
  uint32_t *out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ins = (double)w * iters * 24;
  printf("%-26s waves/SIMD=%d: %.3f ns/instr/SIMD\n", name, w, ms * 1e6 / ins);
  (void)hipFree(out);
}

int main() {
  for (int w : {2, 8}) {
    run<0>("add3 distinct banks", w);
    run<1>("add3 same bank", w);
    run<2>("bitop3 distinct banks", w);
    run<3>("bitop3 same bank", w);
    run<12>("bitop3 two in one bank", w);
    run<13>("xor same bank", w);
    run<14>("xor distinct banks", w);
    run<4>("alignbit distinct banks", w);
    run<5>("alignbit same bank", w);
    run<11>("alignbit x,x,const (rotl)", w);
    run<6>("v_lshl_add_u64", w);
    run<7>("v_lshlrev_b64", w);
    run<8>("v_pk_mov_b32", w);
    run<9>("v_mov_b32", w);
    run<10>("v_add_co_u32", w);
  }
  return 0;
}
