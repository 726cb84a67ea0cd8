"""Debug: where does a sharded run with architecture mutations leave the
unsharded one?  Runs tests/test_sharded_population_gpu.py's workload at
world 1 and 2 and prints per-agent checkpoints."""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _worker(rank, world, out_dir, port):
    import test_sharded_population_gpu as T
    import importlib

    top = importlib.import_module("agilerl_amd.training.train_on_policy")
    from agilerl_amd.population import engine as E

    log = []
    orig_mut = top.mutate_population

    def mut(m, pop, pre_training_mut=False):
        out = orig_mut(m, pop, pre_training_mut=pre_training_mut)
        log.append(("mut", [(a.index, a.mut, a.spec.shape_key()[2:7], a.learn_step, int(a.batch_size),
                             int(a.update_epochs)) for a in out]))
        return out

    top.mutate_population = mut
    orig_train = E.PopulationEngine.train

    def train(self, evo_steps, on_iteration=None):
        pre = [float(v.population.params.data[v.row].double().sum()) for v in self.views]
        out = orig_train(self, evo_steps, on_iteration)
        post = [float(v.population.params.data[v.row].double().sum()) for v in self.views]
        log.append(("train", pre, post, [(g.slots, g.pop.T, g.pop.act_counter) for g in self.groups]))
        return out

    E.PopulationEngine.train = train
    T._run(world, rank, out_dir, port, 0.4)
    torch.save(log, os.path.join(out_dir, f"log_w{world}_r{rank}.pt"))


if __name__ == "__main__":
    out = os.path.join(ROOT, "gpurun_out", "shard_dbg")
    os.makedirs(out, exist_ok=True)
    import socket

    for world in (1, 2):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.start_processes(_worker, args=(world, out, port), nprocs=world, join=True, start_method="spawn")
    logs = {w: [torch.load(os.path.join(out, f"log_w{w}_r{r}.pt"), weights_only=False) for r in range(w)]
            for w in (1, 2)}
    for i, ent in enumerate(logs[1][0]):
        print("W1", ent)
        for r in range(2):
            if i < len(logs[2][r]):
                print(f"W2r{r}", logs[2][r][i])
