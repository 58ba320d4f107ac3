"""Data-loader factory (reference utils/dataset.py:13-116).

``importlib(cfg.data.type).Dataset``; ``DistributedSampler`` when a process
group is initialised (validation/test of video datasets stay
non-distributed, like the reference); pinned memory; ``drop_last`` for train.
"""
import torch
import torch.distributed as dist

from imaginaire_amd.registry import canonical_module_name, import_module


def _get_train_and_val_dataset_objects(cfg):
    dataset_module = import_module(cfg.data.type)
    train_dataset = dataset_module.Dataset(cfg, is_inference=False)
    if hasattr(cfg.data, 'val_type'):
        dataset_module = import_module(cfg.data.val_type)
    val_dataset = dataset_module.Dataset(cfg, is_inference=True)
    return train_dataset, val_dataset


def _get_data_loader(cfg, dataset, batch_size, not_distributed=False, shuffle=True,
                     drop_last=True, seed=0):
    num_workers = getattr(cfg.data, 'num_workers', 8)
    if dist.is_available() and dist.is_initialized() and not not_distributed:
        sampler = torch.utils.data.distributed.DistributedSampler(dataset, seed=seed,
                                                                  shuffle=shuffle)
    elif shuffle:
        sampler = torch.utils.data.RandomSampler(dataset)
    else:
        sampler = torch.utils.data.SequentialSampler(dataset)
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=False,
                                       pin_memory=torch.cuda.is_available(), sampler=sampler,
                                       num_workers=num_workers, drop_last=drop_last,
                                       persistent_workers=num_workers > 0)


def get_train_and_val_dataloader(cfg, seed=0):
    train_dataset, val_dataset = _get_train_and_val_dataset_objects(cfg)
    train_data_loader = _get_data_loader(cfg, train_dataset, cfg.data.train.batch_size,
                                         drop_last=True, seed=seed)
    not_distributed = getattr(cfg.data, 'val_data_loader_not_distributed', False)
    not_distributed = 'video' in canonical_module_name(cfg.data.type) or not_distributed
    val_bs = getattr(getattr(cfg.data, 'val', None), 'batch_size', cfg.data.train.batch_size)
    val_data_loader = _get_data_loader(cfg, val_dataset, val_bs, not_distributed,
                                       shuffle=False, drop_last=getattr(cfg.data.val,
                                                                        'drop_last', False)
                                       if hasattr(cfg.data, 'val') else False, seed=seed)
    return train_data_loader, val_data_loader


def _get_test_dataset_object(cfg):
    dataset_module = import_module(cfg.test_data.type)
    return dataset_module.Dataset(cfg, is_inference=True, is_test=True)


def get_test_dataloader(cfg):
    test_dataset = _get_test_dataset_object(cfg)
    not_distributed = getattr(cfg.test_data, 'val_data_loader_not_distributed', False)
    not_distributed = 'video' in canonical_module_name(cfg.test_data.type) or not_distributed
    return _get_data_loader(cfg, test_dataset, cfg.test_data.test.batch_size, not_distributed,
                            shuffle=False)
