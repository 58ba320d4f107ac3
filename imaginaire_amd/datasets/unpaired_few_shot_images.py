"""Few-shot unpaired image dataset for FUNIT / COCO-FUNIT
(reference datasets/unpaired_few_shot_images.py:10-181): a content image
and a style image with their class indices; evaluation iterates one style
class at a time with a deterministic content stride."""
import random

from imaginaire_amd.datasets.base import BaseDataset
from imaginaire_amd.datasets.images import class_mapping, load_unpaired


class Dataset(BaseDataset):
    def __init__(self, cfg, is_inference=False, is_test=False):
        super().__init__(cfg, is_inference, is_test)
        self.num_content_classes = len(self.class_name_to_idx['images_content'])
        self.num_style_classes = len(self.class_name_to_idx['images_style'])
        self.sample_class_idx = None
        self.content_offset = 8888
        self.content_interval = 100

    def set_sample_class_idx(self, class_idx=None):
        self.sample_class_idx = class_idx
        if class_idx is None:
            self.epoch_length = max(len(v) for v in self.mapping.values())
        else:
            self.epoch_length = len(self.mapping_class['images_style'][class_idx])

    def _create_mapping(self):
        self.mapping, self.epoch_length = class_mapping(self)
        return self.mapping, self.epoch_length

    def _sample_keys(self, index):
        content = self.mapping['images_content']
        if self.is_inference:
            if self.sample_class_idx is None:
                # no class selected (plain ``inference.py``): walk every style image once
                style = self.mapping['images_style'][index % len(self.mapping['images_style'])]
                cls = style['class_idx']
            else:
                cls = self.sample_class_idx
                style = self.mapping_class['images_style'][cls][index]
            ci = ((index + self.content_offset * cls) * self.content_interval) % len(content)
            return {'images_content': content[ci], 'images_style': style}
        return {'images_content': random.choice(content),
                'images_style': random.choice(self.mapping['images_style'])}

    def __getitem__(self, index):
        per_type = self._sample_keys(index)
        data = load_unpaired(self, per_type)
        data['labels_content'] = per_type['images_content']['class_idx']
        data['labels_style'] = per_type['images_style']['class_idx']
        return data
