"""Process "images" for the kflite kubelet (SURVEY.md §2.4, L1 image contract).

The reference ships container images (components/example-notebook-servers); the embedded node
runtime runs pods as process groups, so every image resolves to a process recipe
(native/node/kubelet.cc kDefaultRecipes). These modules honour the same contract as the real
images: HTTP on the container port, the NB_PREFIX base URL, the Jupyter /api/kernels and
/api/terminals endpoints used by the culler, $HOME on the workspace volume.
"""
