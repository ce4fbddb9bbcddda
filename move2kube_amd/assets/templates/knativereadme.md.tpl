Move2Kube
---------
The generated artifacts in this directory move all your application components to Knative. Use them to deploy your application in a Knative instance.

Prerequisites
-------------
* Docker
* Kubectl

Next Steps
----------
{{if .NewImages -}}
* Copy this directory into your base source directory, so that the scripts gets merged at the right contexts.
* Build your images using buildimages.sh
* Push images to registry pushimages.sh
{{end -}}
* Use deploy.sh to deploy your artifacts into a knative.
