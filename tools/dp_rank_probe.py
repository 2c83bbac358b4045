"""Diagnostic: bench's graph-mode DP step with two ranks on one GPU (gloo),
as tests/test_gpu_dist_graphs.py runs it; reports which parameters and
reduced gradients differ between the ranks after each step."""
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import test_gpu_dist_graphs as T  # noqa: E402


def worker(rank, world, port, out, precision):
    T._init(rank, world, port)
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.step import TrainStep

    dev = torch.device("cuda", 0)
    model = T._model(T.DP_SPEC, dev)
    images, targets, ctx = T._data(rank, dev)
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=True, world=world, lr=1e-3,
                     precision=precision, targets=targets, num_boxes=T.NB)
    rec = []
    for it in range(3):
        step(images, ctx, targets, T.NB)
        torch.cuda.synchronize()
        g = {n: v.float().cpu().clone() for n, v in zip([n for n, p in model.named_parameters()
                                                            if any(p is q for q in step.dp_params)],
                                                           step.reducer.views)}
        w = {n: p.detach().float().cpu().clone() for n, p in model.named_parameters()}
        rec.append({"g": g, "w": w, "coef": step.opt.coef.cpu().clone()})
    torch.save(rec, Path(out) / f"r{rank}.pt")
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    prec = sys.argv[1] if len(sys.argv) > 1 else "amp"
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(worker, args=(2, T._port(), d, prec), nprocs=2, join=True, start_method="spawn")
        r0, r1 = torch.load(Path(d) / "r0.pt"), torch.load(Path(d) / "r1.pt")
    for it, (a, b) in enumerate(zip(r0, r1)):
        gd = [(n, float((a["g"][n] - b["g"][n]).abs().max())) for n in a["g"] if not torch.equal(a["g"][n], b["g"][n])]
        wd = [(n, float((a["w"][n] - b["w"][n]).abs().max())) for n in a["w"] if not torch.equal(a["w"][n], b["w"][n])]
        print(f"step {it}: coef {a['coef'].tolist()} vs {b['coef'].tolist()}; grads differ {len(gd)} {gd[:5]}; "
              f"weights differ {len(wd)} {wd[:5]}", flush=True)
