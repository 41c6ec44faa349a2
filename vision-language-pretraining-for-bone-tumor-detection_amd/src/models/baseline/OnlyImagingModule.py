"""OnlyImagingModule (reference src/models/baseline/OnlyImagingModule.py:35-106): the
imaging-only baseline that configs/train.yaml names as its default model.  It is
outside the MI355X hot path (out of scope); the built
downstream module is FusionModule (configs/model/fusion.yaml),
and the pretraining module is VisionLanguageModule
(experiment=pretrain/pretrain_resnet34_tinybert[_mi355x])."""


class OnlyImagingModule:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "OnlyImagingModule is not part of the MI355X build (SURVEY §2 row 15). Run an experiment that "
            "selects a built module, e.g. experiment=pretrain/pretrain_resnet34_tinybert or "
            "experiment=baseline_imaging_and_clinical/baseline_imaging_and_clinical_resnet_34")
