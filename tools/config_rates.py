"""Secondary per-config training rates alone (bench.config_rates): python tools/config_rates.py"""
import json, sys
sys.argv = ['bench']
sys.path.insert(0, '.')
import torch
import bench
r = bench.config_rates(torch.device('cuda'))
print(json.dumps({k: v for k, v in r.items() if 'poisson' in k or 'hypernet' in k or 'sdf' in k}))
