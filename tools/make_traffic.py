"""Turn a tools/pmc_summary.py summary.json into profiles/rNN/pmc_traffic_<config>.json for
bench.py.  Usage: make_traffic.py SUMMARY OUT CONFIG [DTYPE VIEWS_PER_GPU [lists]]

HBM bytes per launch (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB
per dispatch, collected in separate passes; traffic = FETCH_SIZE x 2 + WRITE_SIZE (gfx950's
FETCH_SIZE tallies half the bytes of a read; WRITE_SIZE is exact).  bench.py recomputes the
same sum from the raw KiB stored here."""
import json
import sys

# device kernel (rocprof name, template arguments stripped) -> profiling slot name used by
# bench.py (kd_capi.cpp KernelId)
SLOT = {
    'kd::kd_raster_fwd_pairs': 'kd_raster_fwd', 'kd::kd_raster_fwd': 'kd_raster_fwd',
    'kd::kd_soft_fwd': 'kd_soft_fwd', 'kd::kd_soft_pairs': 'kd_soft_pairs',
    'kd::kd_soft_bwd_items': 'kd_soft_bwd_pairs', 'kd::kd_soft_bwd_pairs': 'kd_soft_bwd_pairs',
    'kd::kd_soft_bwd_lists': 'kd_soft_bwd_pairs',
    'kd::kd_raster_bwd_tile': 'kd_raster_bwd_tile', 'kd::kd_soft_pair_math': 'kd_soft_pair_math',
    'kd::kd_soft_reduce': 'kd_soft_reduce', 'kd::kd_soft_lists': 'kd_soft_reduce',
    'kd::kd_prepare_fwd': 'kd_prepare_fwd', 'kd::kd_prepare_bwd': 'kd_prepare_bwd',
    'kd::kd_zero2': 'kd_zero', 'kd::kd_bin_count': 'kd_bin_count', 'kd::kd_bin_scan': 'kd_bin_scan',
    'kd::kd_bin_scatter': 'kd_bin_scatter', 'kd::kd_soft_ovf_fwd': 'kd_soft_ovf_fwd',
    'kd::kd_soft_ovf_bwd': 'kd_soft_ovf_bwd', 'kd::kd_dibr_bwd': 'kd_dibr_bwd',
    'kd::kd_dibr_fwd_tiles': 'kd_dibr_fwd', 'kd::kd_dibr_fwd_tiles_f64': 'kd_dibr_fwd',
    'kd::kd_dibr_fwd_st': 'kd_dibr_fwd',
}


# per-type VALU instruction counters (tools/pmc_mix.sh); bench.py weights them by issue cost
VALU_MIX = tuple(f'SQ_INSTS_VALU_{k}' for k in (
    'ADD_F32', 'MUL_F32', 'FMA_F32', 'TRANS_F32', 'ADD_F64', 'MUL_F64', 'FMA_F64', 'TRANS_F64',
    'INT32', 'INT64', 'CVT'))


def main(summary, out, config, dtype='f32', views=8, lists=False):
    src = json.load(open(summary))
    kern = {}
    # several device variants can share a slot (e.g. kd_bin_count<.., PREP> of the bench step and
    # the plain kd_bin_count of bench.py's one pair-count call): the slot takes the variant with
    # the most dispatches, i.e. the one the timed step runs
    best = {}
    for name, m in src.items():
        slot = SLOT.get(name.split('<')[0].split('(')[0].replace('void ', ''))
        if slot is None or 'hbm_bytes_raw' not in m:
            continue
        if slot not in best or m.get('dispatches', 0) > src[best[slot]].get('dispatches', 0):
            best[slot] = name
    for slot, name in best.items():
        m = src[name]
        kern[slot] = {'device_kernel': name,
                      'hbm_bytes_per_launch': round(m['hbm_bytes_fetch_x2']),
                      'FETCH_SIZE_KiB': m['FETCH_SIZE'], 'WRITE_SIZE_KiB': m['WRITE_SIZE']}
        kern[slot]['dispatches'] = m.get('dispatches')
        for c in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_WAVES', 'GRBM_GUI_ACTIVE',
                  'SQ_ACTIVE_INST_VALU', 'SQ_INSTS_LDS', 'SQ_WAVE_CYCLES', 'SQ_WAIT_ANY') + VALU_MIX:
            if c in m:  # per launch (bench.py: VALU issue fraction)
                kern[slot][c] = m[c]
    json.dump({'config': config, 'dtype': dtype, 'views_per_gpu': views, 'lists': lists,
               'source': summary, 'traffic': 'FETCH_SIZE x 2 + WRITE_SIZE (KiB x 1024)',
               'kernels': kern}, open(out, 'w'), indent=1)
    print(json.dumps(kern, indent=1))


if __name__ == '__main__':
    a = sys.argv[1:]
    main(a[0], a[1], a[2] if len(a) > 2 else 'c3', a[3] if len(a) > 3 else 'f32',
         int(a[4]) if len(a) > 4 else 8, len(a) > 5 and a[5] == 'lists')
