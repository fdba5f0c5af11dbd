import sys, numpy as np
sys.path.insert(0, 'mcp-raytracer_amd')
import raytracer_amd as rt
sd = rt.generate_scene_data({'type': 'cornell'})
outs = {}
for p in ['ref', 'fp32']:
    cam = rt.create_camera_from_scene_data(sd, {'width': 48, 'samples': 32, 'depth': 16, 'aTolerance': 0, 'precision': p})
    rgb = np.zeros((48, 48, 3), np.uint8); rad = np.zeros((48, 48, 3), np.float32)
    st = cam.render(rgb, radiance=rad)
    outs[p] = rad
    print(p, cam.precision, rad.mean(), st.bounces)
d = np.abs(outs['ref'] - outs['fp32'])
print('max diff', d.max(), 'frac exact', (d == 0).all(-1).mean())
