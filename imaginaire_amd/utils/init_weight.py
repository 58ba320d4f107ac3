"""Weight initialisation (reference utils/init_weight.py:8-61)."""
from torch.nn import init


def weights_init(init_type='normal', gain=0.02, bias=None):
    def init_func(m):
        class_name = m.__class__.__name__
        if hasattr(m, 'weight') and (class_name.find('Conv') != -1 or
                                     class_name.find('Linear') != -1 or
                                     class_name.find('Embedding') != -1):
            weight = getattr(m, 'weight_orig', None)
            if weight is None:
                weight = m.weight
            if init_type == 'normal':
                init.normal_(weight.data, 0.0, gain)
            elif init_type == 'xavier':
                init.xavier_normal_(weight.data, gain=gain)
            elif init_type == 'xavier_uniform':
                init.xavier_uniform_(weight.data, gain=1.0)
            elif init_type == 'kaiming':
                init.kaiming_normal_(weight.data, a=0, mode='fan_in')
            elif init_type == 'orthogonal':
                init.orthogonal_(weight.data, gain=gain)
            elif init_type == 'none':
                m.reset_parameters()
            else:
                raise NotImplementedError('initialization method [%s] is not implemented'
                                          % init_type)
            if hasattr(m, 'bias') and m.bias is not None:
                if bias is not None:
                    bias_type = getattr(bias, 'type', 'normal')
                    if bias_type == 'normal':
                        init.normal_(m.bias.data, 0.0, getattr(bias, 'gain', 0.5))
                    else:
                        raise NotImplementedError('initialization method [%s] is not '
                                                  'implemented' % bias_type)
                else:
                    init.constant_(m.bias.data, 0.0)
    return init_func
