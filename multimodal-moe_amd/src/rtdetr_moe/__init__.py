"""The build's RT-DETR-MoE engine (backbone, hybrid encoder, decoder, loss,
train/val loops) behind src/models/vision/rtdetr.py."""
