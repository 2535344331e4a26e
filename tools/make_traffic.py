"""Turn a tools/pmc_summary.py summary.json into profiles/pmc_traffic.json for bench.py.

HBM bytes per launch (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB
per dispatch, collected in separate passes; the gfx950 FETCH_SIZE x2 correction applies to wide
(16 B/lane) streaming reads only -- our kernels read 4-8 B per lane scattered through L2, so the
raw figure is used as `traffic` and the x2 variant is kept beside it."""
import json
import sys

# device kernel (rocprof name) -> profiling slot name used by bench.py (kd_capi.cpp KernelId)
SLOT = {
    'kd::kd_raster_fwd_pairs': 'kd_raster_fwd', 'kd::kd_raster_fwd<float>': 'kd_raster_fwd',
    'kd::kd_soft_fwd<float, false>': 'kd_soft_fwd', 'kd::kd_soft_fwd<float, true>': 'kd_soft_fwd',
    'kd::kd_soft_pairs<float>': 'kd_soft_pairs',
    'kd::kd_soft_pairs<float, true, 6>': 'kd_soft_pairs',
    'kd::kd_soft_pairs<float, false, 8>': 'kd_soft_pairs',
    'kd::kd_soft_bwd_items<float, 1>': 'kd_soft_bwd_pairs',
    'kd::kd_raster_bwd_tile<float, 3>': 'kd_raster_bwd_tile',
    'kd::kd_soft_pair_math<float, true, false>': 'kd_soft_pair_math',
    'kd::kd_soft_reduce<float>': 'kd_soft_reduce',
    'kd::kd_soft_bwd_pairs<float>': 'kd_soft_bwd_pairs',
    'kd::kd_prepare_fwd<float>': 'kd_prepare_fwd', 'kd::kd_prepare_bwd<float>': 'kd_prepare_bwd',
    'kd::kd_zero2<float>': 'kd_zero',
    'kd::kd_raster_bwd_tile<float, 4>': 'kd_raster_bwd_tile',
    'kd::kd_bin_count<float>': 'kd_bin_count', 'kd::kd_bin_scan': 'kd_bin_scan',
    'kd::kd_bin_scatter<float>': 'kd_bin_scatter',
    'kd::kd_dibr_bwd<float>': 'kd_dibr_bwd',
    'kd::kd_dibr_fwd_tiles': 'kd_dibr_fwd',
    'kd::kd_dibr_fwd_tiles<false>': 'kd_dibr_fwd',
}


def main(summary, out, config, lists=False):
    src = json.load(open(summary))
    kern = {}
    for name, m in src.items():
        slot = SLOT.get(name)
        if slot is None or 'hbm_bytes_raw' not in m:
            continue
        kern[slot] = {'device_kernel': name, 'hbm_bytes_per_launch': round(m['hbm_bytes_raw']),
                      'hbm_bytes_fetch_x2': round(m['hbm_bytes_fetch_x2']),
                      'FETCH_SIZE_KiB': m['FETCH_SIZE'], 'WRITE_SIZE_KiB': m['WRITE_SIZE']}
    json.dump({'config': config, 'lists': lists, 'source': summary, 'kernels': kern},
              open(out, 'w'), indent=1)
    print(json.dumps(kern, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else 'c3')
