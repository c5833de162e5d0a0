"""Debug: 3-rank wheel (hub, lagrangian, xhatshuffle) with the xhat spoke's candidates,
statuses and PDHG iterations printed (GPU; ranks share cuda:0 over gloo)."""
import os, sys, socket
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd")); sys.path.insert(0, ROOT)


def worker(rank, world, port):
    from types import SimpleNamespace
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
    import torch, torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.spin_the_wheel import WheelSpinner
    from mpisppy_amd.utils import cfg_vanilla as vanilla
    from mpisppy_amd.extensions import xhatbase
    orig = xhatbase.XhatBase._try_one

    def spy(self, snamedict, **kw):
        o = orig(self, snamedict, **kw)
        e = self.opt.engine
        print(f"[xhat r{rank}] cand {snamedict} table {getattr(self, 'last_table', None)} obj {o} "
              f"status {e.host('status')} iters {e.host('iters')} wid {self.opt.spcomm.remote_write_id}", flush=True)
        return o
    xhatbase.XhatBase._try_one = spy
    import time
    from mpisppy_amd.cylinders import transport as tp
    og, oa, orr = tp.SpokePort.get, tp.HubPort.answer, tp.HubPort.ready
    t00 = time.perf_counter()

    def get(self, *a):
        t = time.perf_counter()
        r = og(self, *a)
        print(f"[get r{rank}] {t - t00:.4f} -> {time.perf_counter() - t00:.4f} wid {r[3]}", flush=True)
        return r

    def answer(self, *a):
        print(f"[ans r{rank} {self.req_key}] {time.perf_counter() - t00:.4f} wid {a[3]}", flush=True)
        return oa(self, *a)
    cnt = {}

    def ready(self):
        r = orr(self)
        cnt[(self.req_key, r)] = cnt.get((self.req_key, r), 0) + 1
        return r
    tp.SpokePort.get, tp.HubPort.answer, tp.HubPort.ready = get, answer, ready
    import atexit
    atexit.register(lambda: print(f"[ready counts r{rank}] {cnt}", flush=True))
    names = farmer.scenario_names_creator(3)
    cfg = SimpleNamespace(solver_name="mi355x_pdhg", default_rho=1.0, max_iterations=300, rel_gap=1e-4,
                          intra_hub_conv_thresh=1e-10, device="cuda:0", toc=False)
    kw = {"num_scens": 3}
    hub = vanilla.ph_hub(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw)
    spokes = [vanilla.lagrangian_spoke(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw),
              vanilla.xhatshuffle_spoke(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw)]
    ws = WheelSpinner(hub, spokes)
    ws.spin()
    print(f"rank {rank}: inner {ws.BestInnerBound} outer {ws.BestOuterBound} ready counts {cnt}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(worker, args=(3, port), nprocs=3, join=True)
