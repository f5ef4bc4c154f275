"""Builds var/stamp.so, the diagnostic stamp build of the variable-length gate read by tools/probes/stamps.py
(round 6, not product code): s_memtime stamps at the loop top, after the next record, after the first
line, before the finish and at the end of each set; lane 0 stores the clocks per set in a debug array
(ufc_dbg_read).  Usage: python tools/probes/stamp_variant.py stamp"""
import subprocess, sys
subs = [
 # debug buffer + macro
 ('frame_crc_varlen8.hip:namespace ufc_dev {\n\n// Structured buffer load',
  'namespace ufc_dev {\n__device__ uint32_t ufc_dbg_st[1250016 * 8];\n#define UFC_STAMP(t) do { __builtin_amdgcn_sched_barrier(0); unsigned long long t64_; asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t64_) :: "memory"); t = (uint32_t)t64_; __builtin_amdgcn_sched_barrier(0); } while (0)\n\n// Structured buffer load'),
 ('frame_crc_varlen8.hip:  while (QG != kNoSet) {\n    // the next set: geometry from its record; the record after it\n',
  '  while (QG != kNoSet) {\n    uint32_t dbg_t0, dbg_t1, dbg_t3;\n    UFC_STAMP(dbg_t0);\n    // the next set: geometry from its record; the record after it\n'),
 ('frame_crc_varlen8.hip:    O = load_rec(QO);\n    __builtin_amdgcn_sched_barrier(0);\n    auto issue',
  '    O = load_rec(QO);\n    __builtin_amdgcn_sched_barrier(0);\n    UFC_STAMP(dbg_t1);\n    dbg_t2 = dbg_t1;\n    dbg_t1b = dbg_t1;\n    auto issue'),
 ('frame_crc_varlen8.hip:    const uint32_t e = ((zo + 3u) >> 2) & 31u, t = (0u - zo) & 3u;\n    const uint32_t crc = ~unshift(group_lin8_rot(L, c, e), t);',
  '    UFC_STAMP(dbg_t2);\n    const uint32_t e = ((zo + 3u) >> 2) & 31u, t = (0u - zo) & 3u;\n    const uint32_t crc = ~unshift(group_lin8_rot(L, c, e), t);'),
 ('frame_crc_varlen8.hip:      slow_set(QG);\n    }\n    __builtin_amdgcn_sched_barrier(0);\n    QG = QN;',
  '      slow_set(QG);\n    }\n    __builtin_amdgcn_sched_barrier(0);\n    UFC_STAMP(dbg_t3);\n    if (L.lane == 0u && QG < 1250016u) { *(uint4*)(ufc_dbg_st + (uint64_t)QG * 8) = make_uint4(dbg_t0, dbg_t1, dbg_t2, dbg_t3); *(uint4*)(ufc_dbg_st + (uint64_t)QG * 8 + 4) = make_uint4(dbg_t1b, M.slow ? 1u : 0u, 0u, 0u); }\n    QG = QN;'),
 ('frame_crc_varlen8.hip:      c = Chains{x.x, x.y, x.z, x.w, 0u};\n      if (s > 0) issue(s, &c);\n    };',
  '      c = Chains{x.x, x.y, x.z, x.w, 0u};\n      if (s > 0) issue(s, &c);\n      UFC_STAMP(dbg_t1b);\n    };'),
 ('frame_crc_varlen8.hip:  Lane8 L;\n  init_lane8(L, lds, p.G);\n  const uint64_t nfr', '  Lane8 L;\n  init_lane8(L, lds, p.G);\n  uint32_t dbg_t2 = 0, dbg_t1b = 0;\n  const uint64_t nfr'),
 ('frame_crc_varlen8.hip:int varlen8_waves() { return kV8Waves; }',
  'int varlen8_waves() { return kV8Waves; }\n}  // namespace ufc_dev\nextern "C" int ufc_dbg_read(void* dst) { return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ufc_dev::ufc_dbg_st), sizeof(ufc_dev::ufc_dbg_st), 0, hipMemcpyDeviceToHost); }\nnamespace ufc_dev {'),
]
args = [sys.executable, "tools/build_variant.py", sys.argv[1]] + [a + "=>" + b for a, b in subs]
sys.exit(subprocess.run(args).returncode)
