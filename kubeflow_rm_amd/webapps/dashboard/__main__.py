from kubeflow_rm_amd.webapps.dashboard import create_app, serve

if __name__ == "__main__":
    serve(create_app())
