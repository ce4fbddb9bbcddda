#   Copyright IBM Corporation 2020
#
#   Licensed under the Apache License, Version 2.0 (the "License");
#   you may not use this file except in compliance with the License.
#   You may obtain a copy of the License at
#
#        http://www.apache.org/licenses/LICENSE-2.0
#
#   Unless required by applicable law or agreed to in writing, software
#   distributed under the License is distributed on an "AS IS" BASIS,
#   WITHOUT WARRANTIES OR CONDITIONS OF ANY KIND, either express or implied.
#   See the License for the specific language governing permissions and
#   limitations under the License.

# Invoke as pushimages.sh <registry_url> <registry_namespace>

if [ "$#" -ne 2 ]; then
    REGISTRY_URL=docker.io
    REGISTRY_NAMESPACE=myproject
else
    REGISTRY_URL=$1
    REGISTRY_NAMESPACE=$2
fi

# Uncomment the below line if you want to enable login before pushing
# docker login ${REGISTRY_URL}

docker tag myproject-docker-compose-api:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-docker-compose-api:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-docker-compose-api:latest
docker tag myproject-docker-compose-web:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-docker-compose-web:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-docker-compose-web:latest
docker tag myproject-dockerfile:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-dockerfile:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/myproject-dockerfile:latest
docker tag fibonacci-api:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/fibonacci-api:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/fibonacci-api:latest
docker tag fibonacci-web:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/fibonacci-web:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/fibonacci-web:latest
docker tag docker-compose:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/docker-compose:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/docker-compose:latest
docker tag dockerfile:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/dockerfile:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/dockerfile:latest
docker tag golang:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/golang:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/golang:latest
docker tag java-gradle:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-gradle:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-gradle:latest
docker tag java-maven:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-maven:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-maven:latest
docker tag nodejs:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/nodejs:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/nodejs:latest
docker tag php:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/php:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/php:latest
docker tag python:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/python:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/python:latest
docker tag ruby:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/ruby:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/ruby:latest
