"""Base GAN trainer (reference trainers/base.py:27-829).

Keeps the reference's hooks and semantics — loss registry (``criteria`` /
``weights`` / ``gen_losses`` / ``dis_losses``), requires_grad toggling,
``dis_step``/``gen_step``, EMA update after the G step, iteration/epoch LR
policies, meters, image dumps, ``speed_benchmark`` phase timers, FID-based
``best_FID``, checkpoint file naming and dictionary keys, auto-resume through
``latest_checkpoint.txt`` — with an MI355X step:

* bf16 autocast instead of apex AMP (no loss scaler, no fp16 master copies);
* inputs moved to the GPU as channels-last (NHWC) tensors;
* gradients synchronised by the bucketed RCCL DDP with backward overlap
  (``begin()`` before, ``finish()`` after each backward);
* losses stay on the device; host synchronisation happens only at logging
  boundaries (the reference calls ``.item()`` every logging iteration too, but
  also forces device syncs in ``speed_benchmark`` mode — kept, opt-in).
"""
import contextlib
import os
import time

import torch
from torch import nn

from imaginaire_amd.utils import trace
from imaginaire_amd.utils.distributed import is_master, master_only
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.io import save_pilimage_in_jpeg
from imaginaire_amd.utils.meters import Meter, add_hparams
from imaginaire_amd.utils.misc import requires_grad, to_device
from imaginaire_amd.utils.model_average import calibrate_batch_norm_momentum, reset_batch_norm
from imaginaire_amd.utils.visualization.common import save_image_grid, tensor2pilimage


def amp_dtype_of(cfg, device):
    amp = getattr(cfg.trainer, 'amp', 'O0')
    if device.type != 'cuda':
        return None
    if amp in ('O1', 'O2', 'O3', 'bf16', True):
        return torch.bfloat16
    return None


class BaseTrainer(object):
    # True when every rank runs the same sequence of network calls each iteration (no
    # data-dependent sub-networks): DDP then uses its rank-local unused-parameter mask (no host
    # sync per backward) and the multi-rank step can be captured into a hipGraph
    # (utils/trainer.py _find_unused_mode, utils/cuda_graph.py graph_supported)
    rank_uniform_control_flow = False

    @classmethod
    def rank_uniform(cls, cfg):
        """Whether THIS configuration's iteration is rank-uniform (see above); families whose
        uniformity depends on the config (the vid2vid family's optional hand discriminator)
        override it. Read before the trainer exists (utils/trainer.py wraps the networks
        first)."""
        return cls.rank_uniform_control_flow

    def __init__(self, cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, train_data_loader,
                 val_data_loader):
        super().__init__()
        print('Setup trainer.')
        self.cfg = cfg
        self.rank_uniform_control_flow = type(self).rank_uniform(cfg)
        self.net_G = net_G
        if cfg.trainer.model_average:
            self.net_G_module = self.net_G.module.module
        else:
            self.net_G_module = self.net_G.module
        self.val_data_loader = val_data_loader
        self.is_inference = train_data_loader is None
        self.net_D = net_D
        self.opt_G = opt_G
        self.opt_D = opt_D
        self.sch_G = sch_G
        self.sch_D = sch_D
        self.train_data_loader = train_data_loader
        self.device = next(self.net_G.parameters()).device
        self.amp_dtype = amp_dtype_of(cfg, self.device)
        self.channels_last = self.device.type == 'cuda'
        self.criteria = nn.ModuleDict()
        self.weights = dict()
        self.losses = dict(gen_update=dict(), dis_update=dict())
        self.gen_losses = self.losses['gen_update']
        self.dis_losses = self.losses['dis_update']
        self._init_loss(cfg)
        for loss_name, loss_weight in self.weights.items():
            print("Loss {:<20} Weight {}".format(loss_name, loss_weight))
        self.criteria.to(self.device)
        for crit in self.criteria.values():
            if hasattr(crit, 'to_device_format') and self.device.type == 'cuda':
                crit.to_device_format()
        if self.is_inference:
            return
        self.current_iteration = 0
        self.current_epoch = 0
        self.start_iteration_time = None
        self.start_epoch_time = None
        self.elapsed_iteration_time = 0
        self.time_iteration = -1
        self.time_epoch = -1
        self.best_fid = None
        self.speed_benchmark = getattr(self.cfg, 'speed_benchmark', False)
        self._reset_speed_accumulators()
        self._init_tensorboard()
        self._init_hparams()

    # ------------------------------------------------------------------
    def autocast(self):
        if self.amp_dtype is None:
            return contextlib.nullcontext()
        # no autocast weight-cast cache inside a hipGraph capture (cached casts would be
        # graph-pool tensors outliving the region that produced them)
        return torch.autocast(device_type='cuda', dtype=self.amp_dtype,
                              cache_enabled=not torch.cuda.is_current_stream_capturing())

    def _reset_speed_accumulators(self):
        for k in ('gen_forw', 'gen_loss', 'gen_back', 'gen_step', 'gen_avg', 'dis_forw',
                  'dis_loss', 'dis_back', 'dis_step'):
            setattr(self, 'accu_%s_iter_time' % k, 0)

    def _init_tensorboard(self):
        self.meters = {}
        for name in ['optim/gen_lr', 'optim/dis_lr', 'time/iteration', 'time/epoch']:
            self.meters[name] = Meter(name)
        self.metric_meters = {}
        for name in ['FID', 'best_FID']:
            self.metric_meters[name] = Meter(name)
        self.image_meter = Meter('images')

    def _init_hparams(self):
        self.hparam_dict = {}

    def _write_tensorboard(self):
        self._write_to_meters({'time/iteration': self.time_iteration,
                               'time/epoch': self.time_epoch,
                               'optim/gen_lr': self.sch_G.get_last_lr()[0],
                               'optim/dis_lr': self.sch_D.get_last_lr()[0]}, self.meters)
        self._write_loss_meters()
        self._write_custom_meters()
        self._flush_meters(self.meters)

    def _write_loss_meters(self):
        for update, losses in self.losses.items():
            for loss_name, loss in losses.items():
                full = update + '/' + loss_name
                if full not in self.meters:
                    self.meters[full] = Meter(full)
                self.meters[full].write(loss)

    def _write_custom_meters(self):
        pass

    @staticmethod
    def _write_to_meters(data, meters):
        for key, value in data.items():
            meters[key].write(value)

    def _flush_meters(self, meters):
        for meter in meters.values():
            meter.flush(self.current_iteration)

    # ------------------------------------------------------------------
    def _pre_save_checkpoint(self):
        pass

    def sync_buffers(self):
        """Broadcast rank 0's buffers (BN running stats, SN u/v, EMA copy) to every rank:
        the DDP wrapper does not broadcast them before each forward (the reference's torch
        DDP does), so they are made identical wherever they are observed — checkpoints and
        evaluation."""
        _ddp_call(self.net_G, 'sync_buffers')
        if self.net_D is not None:
            _ddp_call(self.net_D, 'sync_buffers')

    def save_checkpoint(self, current_epoch, current_iteration):
        self.sync_buffers()
        self._pre_save_checkpoint()
        return _save_checkpoint(self.cfg, self.net_G, self.net_D, self.opt_G, self.opt_D,
                                self.sch_G, self.sch_D, current_epoch, current_iteration)

    def load_checkpoint(self, cfg, checkpoint_path, resume=None):
        if checkpoint_path is not None and os.path.exists(checkpoint_path):
            if resume is None:
                resume = False
        elif os.path.exists(os.path.join(cfg.logdir, 'latest_checkpoint.txt')):
            fn = os.path.join(cfg.logdir, 'latest_checkpoint.txt')
            with open(fn, 'r') as f:
                line = f.read().splitlines()
            checkpoint_path = os.path.join(cfg.logdir, line[0].split(' ')[-1])
            if resume is None:
                resume = True
        else:
            print('No checkpoint found.')
            return 0, 0
        checkpoint = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
        current_epoch = 0
        current_iteration = 0
        if resume:
            self.net_G.load_state_dict(checkpoint['net_G'])
            if not self.is_inference:
                self.net_D.load_state_dict(checkpoint['net_D'])
                if 'opt_G' in checkpoint:
                    self.opt_G.load_state_dict(checkpoint['opt_G'])
                    self.opt_D.load_state_dict(checkpoint['opt_D'])
                    self.sch_G.load_state_dict(checkpoint['sch_G'])
                    self.sch_D.load_state_dict(checkpoint['sch_D'])
                    current_epoch = checkpoint['current_epoch']
                    current_iteration = checkpoint['current_iteration']
                    print('Load from: {}'.format(checkpoint_path))
                else:
                    print('Load network weights only.')
        else:
            self.net_G.load_state_dict(checkpoint['net_G'])
            print('Load generator weights only.')
        print('Done with loading the checkpoint.')
        return current_epoch, current_iteration

    # ------------------------------------------------------------------
    def start_of_epoch(self, current_epoch):
        self._start_of_epoch(current_epoch)
        self.current_epoch = current_epoch
        self.start_epoch_time = time.time()

    def to_device(self, data):
        return to_device(data, self.device, non_blocking=True,
                         memory_format=torch.channels_last if self.channels_last else None)

    def start_of_iteration(self, data, current_iteration):
        data = self._start_of_iteration(data, current_iteration)
        data = self.to_device(data)
        self.current_iteration = current_iteration
        if not self.is_inference:
            self.net_D.train()
        self.net_G.train()
        self.start_iteration_time = time.time()
        return data

    def end_of_iteration(self, data, current_epoch, current_iteration):
        self.current_iteration = current_iteration
        self.current_epoch = current_epoch
        if self.cfg.gen_opt.lr_policy.iteration_mode:
            self.sch_G.step()
        if self.cfg.dis_opt.lr_policy.iteration_mode:
            self.sch_D.step()
        self.elapsed_iteration_time += time.time() - self.start_iteration_time
        if current_iteration % self.cfg.logging_iter == 0:
            ave_t = self.elapsed_iteration_time / self.cfg.logging_iter
            self.time_iteration = ave_t
            print('Iteration: {}, average iter time: {:6f}.'.format(current_iteration, ave_t))
            self.elapsed_iteration_time = 0
            if self.speed_benchmark:
                n = self.cfg.logging_iter
                for tag, key in (('Generator FWD', 'gen_forw'), ('Generator LOS', 'gen_loss'),
                                 ('Generator BCK', 'gen_back'), ('Generator STP', 'gen_step'),
                                 ('Generator AVG', 'gen_avg'), ('Discriminator FWD', 'dis_forw'),
                                 ('Discriminator LOS', 'dis_loss'),
                                 ('Discriminator BCK', 'dis_back'),
                                 ('Discriminator STP', 'dis_step')):
                    print('\t{} time {:6f}'.format(tag, getattr(self, 'accu_%s_iter_time' % key)
                                                   / n))
                print('{:6f}'.format(ave_t))
                self._reset_speed_accumulators()
        self._end_of_iteration(data, current_epoch, current_iteration)
        if current_iteration >= self.cfg.snapshot_save_start_iter and \
                current_iteration % self.cfg.snapshot_save_iter == 0:
            self.save_image(self._get_save_path('images', 'jpg'), data)
            self.save_checkpoint(current_epoch, current_iteration)
            self.write_metrics()
        elif current_iteration % self.cfg.image_save_iter == 0:
            self.save_image(self._get_save_path('images', 'jpg'), data)
        elif current_iteration % self.cfg.image_display_iter == 0:
            self.save_image(os.path.join(self.cfg.logdir, 'images', 'current.jpg'), data)
        if current_iteration % self.cfg.logging_iter == 0:
            self._write_tensorboard()

    def end_of_epoch(self, data, current_epoch, current_iteration):
        self.current_iteration = current_iteration
        self.current_epoch = current_epoch
        if not self.cfg.gen_opt.lr_policy.iteration_mode:
            self.sch_G.step()
        if not self.cfg.dis_opt.lr_policy.iteration_mode:
            self.sch_D.step()
        elapsed_epoch_time = time.time() - self.start_epoch_time
        print('Epoch: {}, total time: {:6f}.'.format(current_epoch, elapsed_epoch_time))
        self.time_epoch = elapsed_epoch_time
        self._end_of_epoch(data, current_epoch, current_iteration)
        if current_epoch >= self.cfg.snapshot_save_start_epoch and \
                current_epoch % self.cfg.snapshot_save_epoch == 0:
            self.save_image(self._get_save_path('images', 'jpg'), data)
            self.save_checkpoint(current_epoch, current_iteration)
            self.write_metrics()

    def pre_process(self, data):
        pass

    def recalculate_model_average_batch_norm_statistics(self, data_loader):
        if not self.cfg.trainer.model_average:
            return
        n_iter = self.cfg.trainer.model_average_batch_norm_estimation_iteration
        if n_iter == 0 or data_loader is None:
            return
        with torch.no_grad(), self.autocast():
            avg = self.net_G.module.averaged_model
            avg.train()
            avg.apply(reset_batch_norm)
            for cal_it, cal_data in enumerate(data_loader):
                if cal_it >= n_iter:
                    break
                cal_data = self.to_device(self._start_of_iteration(cal_data, 0))
                avg.apply(calibrate_batch_norm_momentum)
                avg(cal_data)

    def save_image(self, path, data):
        self.net_G.eval()
        vis_images = self._get_visualizations(data)
        if is_master() and vis_images is not None:
            vis_images = [v.float() for v in vis_images]
            vis_images = torch.cat(vis_images, dim=3)
            vis_images = ((vis_images + 1) / 2).clamp_(0, 1)
            print('Save output images to {}'.format(path))
            save_image_grid(vis_images, path, nrow=1, padding=0, normalize=True)
            if self.cfg.trainer.image_to_tensorboard:
                # the same grid as the PNG (nrow=1, padding=0: samples stacked vertically)
                grid = torch.cat(list(vis_images), dim=1)
                self.image_meter.write_image(grid, self.current_iteration)
        self.net_G.train()

    def write_metrics(self):
        self.sync_buffers()
        cur_fid = self._compute_fid()
        if cur_fid is not None:
            self.best_fid = cur_fid if self.best_fid is None else min(self.best_fid, cur_fid)
            metric_dict = {'FID': cur_fid, 'best_FID': self.best_fid}
            self._write_to_meters(metric_dict, self.metric_meters)
            self._flush_meters(self.metric_meters)
            if self.cfg.trainer.hparam_to_tensorboard:
                add_hparams(self.hparam_dict, metric_dict)

    def _get_save_path(self, subdir, ext):
        subdir_path = os.path.join(self.cfg.logdir, subdir)
        os.makedirs(subdir_path, exist_ok=True)
        return os.path.join(subdir_path, 'epoch_{:05}_iteration_{:09}.{}'.format(
            self.current_epoch, self.current_iteration, ext))

    def _get_outputs(self, net_D_output, real=True):
        def _diff(a, b):
            out = []
            for x, y in zip(a, b):
                out.append(_diff(x, y) if isinstance(x, list) else x - y)
            return out
        if real:
            if self.cfg.trainer.gan_relativistic:
                return _diff(net_D_output['real_outputs'], net_D_output['fake_outputs'])
            return net_D_output['real_outputs']
        if self.cfg.trainer.gan_relativistic:
            return _diff(net_D_output['fake_outputs'], net_D_output['real_outputs'])
        return net_D_output['fake_outputs']

    def _start_of_epoch(self, current_epoch):
        pass

    def _start_of_iteration(self, data, current_iteration):
        return data

    def _end_of_iteration(self, data, current_epoch, current_iteration):
        pass

    def _end_of_epoch(self, data, current_epoch, current_iteration):
        pass

    def _get_visualizations(self, data):
        return None

    def _compute_fid(self):
        return None

    def _init_loss(self, cfg):
        raise NotImplementedError

    # ------------------------------------------------------------------
    def _sync(self):
        if self.speed_benchmark and self.device.type == 'cuda':
            torch.cuda.synchronize()
        return time.time()

    def gen_update(self, data):
        self.opt_G.zero_grad(set_to_none=True)
        requires_grad(self.net_G_module, True)
        requires_grad(self.net_D, False)
        self.forw_time = self._sync()
        with trace.phase('gen/forward'), self.autocast():
            total_loss = self.gen_forward(data)
        if total_loss is None:
            return
        self.back_time = self._sync()
        with trace.phase('gen/backward'):
            _ddp_call(self.net_G, 'begin')
            total_loss.backward()
            _ddp_call(self.net_G, 'finish')
        if hasattr(self.cfg.gen_opt, 'clip_grad_norm'):
            nn.utils.clip_grad_norm_(self.net_G_module.parameters(),
                                     self.cfg.gen_opt.clip_grad_norm)
        self.step_time = self._sync()
        with trace.phase('gen/step'):
            if self._step_ok(total_loss):
                self.opt_G.step()
        self.avg_time = self._sync()
        if self.cfg.trainer.model_average:
            with trace.phase('gen/ema'):
                self.net_G.module.update_average()
        self._detach_losses()
        self._time_before_leave_gen()

    def gen_forward(self, data):
        raise NotImplementedError

    def dis_update(self, data):
        self.opt_D.zero_grad(set_to_none=True)
        requires_grad(self.net_G_module, False)
        requires_grad(self.net_D, True)
        self.forw_time = self._sync()
        with trace.phase('dis/forward'), self.autocast():
            total_loss = self.dis_forward(data)
        if total_loss is None:
            return
        self.back_time = self._sync()
        with trace.phase('dis/backward'):
            _ddp_call(self.net_D, 'begin')
            total_loss.backward()
            _ddp_call(self.net_D, 'finish')
        self.step_time = self._sync()
        with trace.phase('dis/step'):
            if self._step_ok(total_loss):
                self.opt_D.step()
        self._detach_losses()
        self._time_before_leave_dis()

    def _step_ok(self, total_loss):
        """Optional non-finite-loss guard (``trainer.skip_nonfinite_steps``): the
        bf16 counterpart of apex's dynamic-loss-scale overflow skip. Costs one
        device->host sync per update, so it is off by default."""
        if not getattr(self.cfg.trainer, 'skip_nonfinite_steps', False):
            return True
        ok = bool(torch.isfinite(total_loss.detach()).all())
        if not ok:
            print('Non-finite loss at iteration {}; skipping the optimizer step.'.format(
                self.current_iteration))
        return ok

    def dis_forward(self, data):
        raise NotImplementedError

    def test(self, data_loader, output_dir, inference_args):
        if self.cfg.trainer.model_average:
            net_G = self.net_G.module.averaged_model
        else:
            net_G = self.net_G.module
        net_G.eval()
        print('# of samples %d' % len(data_loader))
        for it, data in enumerate(data_loader):
            data = self.start_of_iteration(data, current_iteration=-1)
            with torch.no_grad(), self.autocast():
                output_images, file_names = net_G.inference(data, **vars(inference_args))
            if isinstance(file_names, str):
                file_names = [file_names]
            for output_image, file_name in zip(output_images, file_names):
                fullname = os.path.join(output_dir, file_name + '.jpg')
                output_image = tensor2pilimage(output_image.float().clamp_(-1, 1),
                                               minus1to1_normalized=True)
                save_pilimage_in_jpeg(fullname, output_image)

    def _get_total_loss(self, gen_forward):
        losses = self.gen_losses if gen_forward else self.dis_losses
        total_loss = torch.zeros((), device=self.device)
        for loss_name in self.weights:
            if loss_name in losses:
                total_loss = total_loss + losses[loss_name] * self.weights[loss_name]
        losses['total'] = total_loss
        return total_loss

    def _detach_losses(self):
        for k in self.gen_losses:
            self.gen_losses[k] = self.gen_losses[k].detach()
        for k in self.dis_losses:
            self.dis_losses[k] = self.dis_losses[k].detach()

    def _time_before_loss(self):
        self.loss_time = self._sync()

    def _time_before_leave_gen(self):
        if self.speed_benchmark:
            end_time = self._sync()
            self.accu_gen_forw_iter_time += self.loss_time - self.forw_time
            self.accu_gen_loss_iter_time += self.back_time - self.loss_time
            self.accu_gen_back_iter_time += self.step_time - self.back_time
            self.accu_gen_step_iter_time += self.avg_time - self.step_time
            self.accu_gen_avg_iter_time += end_time - self.avg_time

    def _time_before_leave_dis(self):
        if self.speed_benchmark:
            end_time = self._sync()
            self.accu_dis_forw_iter_time += self.loss_time - self.forw_time
            self.accu_dis_loss_iter_time += self.back_time - self.loss_time
            self.accu_dis_back_iter_time += self.step_time - self.back_time
            self.accu_dis_step_iter_time += end_time - self.step_time


def _ddp_call(net, fn):
    f = getattr(net, fn, None)
    if f is not None and callable(f):
        f()


@master_only
def _save_checkpoint(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, current_epoch,
                     current_iteration):
    latest_checkpoint_path = 'epoch_{:05}_iteration_{:09}_checkpoint.pt'.format(
        current_epoch, current_iteration)
    save_path = os.path.join(cfg.logdir, latest_checkpoint_path)
    os.makedirs(cfg.logdir, exist_ok=True)
    # written to a temporary name and renamed, pointer file last: a rank killed mid-save
    # (watchdog, lost node) never leaves latest_checkpoint.txt naming a torn file, so the
    # restarted job auto-resumes from the previous complete checkpoint
    torch.save({'net_G': net_G.state_dict(), 'net_D': net_D.state_dict(),
                'opt_G': opt_G.state_dict(), 'opt_D': opt_D.state_dict(),
                'sch_G': sch_G.state_dict(), 'sch_D': sch_D.state_dict(),
                'current_epoch': current_epoch, 'current_iteration': current_iteration},
               save_path + '.tmp')
    os.replace(save_path + '.tmp', save_path)
    pointer = os.path.join(cfg.logdir, 'latest_checkpoint.txt')
    with open(pointer + '.tmp', 'wt') as f:
        f.write('latest_checkpoint: %s' % latest_checkpoint_path)
    os.replace(pointer + '.tmp', pointer)
    print('Save checkpoint to {}'.format(save_path))
    return save_path
