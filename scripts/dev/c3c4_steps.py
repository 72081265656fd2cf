import sys, json, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))); sys.path.insert(0, sys.path[0] + "/kge-1_amd")
import bench
r = bench.other_configs(torch.device("cuda:0"))
print(json.dumps(r))
