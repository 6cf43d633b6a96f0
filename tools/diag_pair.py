"""Diagnostic: device vs oracle ICP per iteration count on one revisit pair."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from lidar_slam_arvc_amd import _lib, synthetic
from oracle import open3d_restated as O

ps = synthetic.make_revisit_pairs(3, seed=41, model=synthetic.VLP16_8K)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 0
dev = _lib.device(0)
ids = [dev.upload(ps.targets[k]), dev.upload(ps.sources[k])]
dev.preprocess(ids, _lib.prep_params())
tgt = O.filter_radius_height(ps.targets[k]); src = O.filter_radius_height(ps.sources[k])
xyz, nrm = dev.download(ids[0], normals=True)
ref_n = O.estimate_normals(tgt)
d = np.abs(np.sum(nrm * ref_n, 1))
print('normals: worst |dot|', np.sort(d)[:5], 'n bad', (d < 1 - 1e-5).sum(), 'of', len(d))
for it in list(range(0, 8)) + [10, 15, 20, 30]:
    g = dev.icp_batch([ids[1]], [ids[0]], ps.init[k:k+1], _lib.icp_params(max_iteration=it))[0]
    gc = dev.last_correspondences()
    r = O.registration_icp(src, tgt, 10.0, ps.init[k], "p2plane", ref_n, max_iteration=it)
    a = {tuple(x) for x in gc.tolist()}; b = {tuple(x) for x in r['correspondences'].tolist()}
    print(it, 'iters', g['iterations'], r['iterations'], 'dT', np.abs(g['transformation'] - r['transformation']).max(),
          'fit', g['fitness'] - r['fitness'], 'rmse', g['inlier_rmse'] - r['inlier_rmse'], 'corr diff', len(a ^ b))
    if len(a ^ b) and it < 3:
        diff = sorted(a ^ b)[:6]; print('   ', diff)
