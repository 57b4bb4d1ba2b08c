import sys; sys.path.insert(0,'tests'); sys.path.insert(0,'optical-flow-using-dense-inverse-search_amd')
import numpy as np, scenes, disflow
for preset in ('MEDIUM','FAST','ULTRAFAST'):
    for seed in (30, 31, 40, 50):
        I0, I1 = scenes.scene_pair(seed, 1920, 1080)
        p = disflow.preset_params(disflow.Preset[preset], 1920, 1080)
        e = disflow.DenseInverseSearch(p, 1920, 1080)
        e.calc(I0, I1)
        print(preset, seed, [e.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)])
I0, I1 = disflow.synth_pair(0, 1920, 1080)
p = disflow.preset_params(disflow.Preset.MEDIUM, 1920, 1080); e = disflow.DenseInverseSearch(p, 1920, 1080); e.calc(I0, I1)
print('synth', [e.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)])
