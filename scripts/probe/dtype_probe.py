"""Print the output dtype of every module of a family's generator under bf16 autocast (finds
where activations fall back to fp32)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    cfg = Config(os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else
                              'configs/unit_test/munit.yaml'))
    cfg.logdir = '/tmp/iamd_dtype_probe'
    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    tr = get_trainer(cfg, *nets, [], None)
    from imaginaire_amd.utils.dataset import get_train_and_val_dataloader
    loader, _ = get_train_and_val_dataloader(cfg)
    data = tr.start_of_iteration(next(iter(loader)), 0)
    seen = []
    for name, m in tr.net_G.named_modules():
        def hook(mod, inp, out, name=name):
            i = inp[0].dtype if inp and torch.is_tensor(inp[0]) else None
            o = out.dtype if torch.is_tensor(out) else None
            seen.append((name, type(mod).__name__, i, o))
        m.register_forward_hook(hook)
    with torch.no_grad(), tr.autocast():
        tr.net_G(data)
    for name, typ, i, o in seen:
        if o == torch.float32 or i == torch.float32:
            print('%-70s %-22s in %s out %s' % (name[-70:], typ, i, o))


if __name__ == '__main__':
    main()
